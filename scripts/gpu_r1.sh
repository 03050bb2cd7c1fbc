#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m arbius_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_hip.log 2>&1 || { tail -30 gpurun_out/bench_hip.log; exit 1; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --reference-ops > gpurun_out/bench_ref.log 2>&1 || { tail -30 gpurun_out/bench_ref.log; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_hip -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_hip.log 2>&1
echo done
