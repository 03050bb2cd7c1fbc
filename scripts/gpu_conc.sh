#!/bin/bash
# Concurrent-task sweep: tasks/hour and p50 vs pipeline forks per GPU (sd15, kandinsky2).
set -o pipefail
TAG=${1:-c1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -m arbius_amd.ops.build > $O/build.log 2>&1 && python -m arbius_amd.native.build >> $O/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for c in 1 2 3 4; do
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --concurrent $c > $O/bench_sd_c$c.log 2>&1 || { tail -20 $O/bench_sd_c$c.log; exit 1; }
  tail -1 $O/bench_sd_c$c.log | cut -c1-200
done
for c in 1 2; do
  timeout -k 10 600 python bench.py --model kandinsky2 --steps 2 --warmup 1 --concurrent $c > $O/bench_k2_c$c.log 2>&1 || { tail -20 $O/bench_k2_c$c.log; exit 1; }
  tail -1 $O/bench_k2_c$c.log | cut -c1-200
done
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_sd -o run -- python3 $R/bench.py --steps 1 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/prof_sd/run_results.db --top 40 --md $O/rocprof_sd.md > /dev/null 2>&1; rm -rf $O/prof_sd
echo done
