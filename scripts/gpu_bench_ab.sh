#!/bin/bash
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m arbius_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python scripts/kernel_ab.py attn > gpurun_out/kernel_ab_$TAG.log 2>&1 || { tail -20 gpurun_out/kernel_ab_$TAG.log; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_$TAG.log 2>&1 || { tail -30 gpurun_out/bench_$TAG.log; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
echo done
