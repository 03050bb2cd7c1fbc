#!/bin/bash
# round 2: family table for solo (ratio 4) and 2-stream lock-step (ratio 1) shapes: GPU tests
# (goldens included), default + latency SD bench, rocprof kernel summary of the default config
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2f3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_sd_default.json 2> $O/bench_sd_default.err || { tail -20 $O/bench_sd_default.err; exit 1; }
cat $O/bench_sd_default.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 1 > $O/bench_sd_latency.json 2> $O/bench_sd_latency.err || { tail -20 $O/bench_sd_latency.err; exit 1; }
cat $O/bench_sd_latency.json
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/p_sd/run_results.db --top 45 --md $O/rocprof_sd15_default.md > /dev/null 2>&1; rm -rf $O/p_sd
head -16 $O/rocprof_sd15_default.md | cut -c1-140
