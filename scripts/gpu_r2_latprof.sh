#!/bin/bash
# round 2: rocprof kernel summary of the SD1.5 latency mode (1 stream, solo tasks) with the family table
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2lat}
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_lat -o run -- python3 $R/bench.py --steps 3 --warmup 1 --concurrent 1 --group 1 > $O/prof_lat.log 2>&1) || { tail -20 $O/prof_lat.log; exit 1; }
python scripts/prof_summary.py $O/p_lat/run_results.db --top 45 --md $O/rocprof_sd15_latency.md > /dev/null 2>&1; rm -rf $O/p_lat
head -30 $O/rocprof_sd15_latency.md | cut -c1-150
