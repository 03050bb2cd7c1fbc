#!/bin/bash
# Kandinsky2 milestone on one MI355X: GPU tests, kandinsky2 + anythingv3 bench, rocprof of kandinsky2.
set -o pipefail
TAG=${1:-k2}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -m arbius_amd.ops.build > $O/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
timeout -k 10 600 python bench.py --model kandinsky2 --steps 1 --warmup 1 > $O/bench_k2.log 2>&1 || { tail -30 $O/bench_k2.log; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model kandinsky2 --steps 1 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/bench_sd.log 2>&1 || { tail -30 $O/bench_sd.log; exit 1; }
cat $O/bench_k2.log | tail -2; tail -1 $O/bench_sd.log
echo done
