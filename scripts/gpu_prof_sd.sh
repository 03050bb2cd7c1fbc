#!/bin/bash
# Attention microbench (in-model layouts) + rocprofv3 kernel stats of the default SD1.5 bench config.
set -o pipefail
TAG=${1:-profsd}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python scripts/microbench.py $O/micro.json > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
grep attention $O/micro.log | cut -c1-200
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/p -o run -- python3 $R/bench.py --steps 2 --warmup 1 ${BENCH_ARGS:-} > $O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log | cut -c1-300
python scripts/prof_summary.py $O/p/run_results.db --top 40 --md $O/rocprof_sd15.md > /dev/null 2>&1; rm -rf $O/p
head -24 $O/rocprof_sd15.md | cut -c1-150
