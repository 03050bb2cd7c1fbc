#!/bin/bash
# round 2 / call B: fused-sampler kernel tests, re-pin goldens (NUMERICS r2.1), bench default + latency mode
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r2b.log 2>&1 || { tail -40 gpurun_out/pytest_r2b.log; exit 1; }
tail -2 gpurun_out/pytest_r2b.log
timeout -k 10 900 python -u scripts/pin_goldens.py --out gpurun_out/golden_r2b.json --selftest > gpurun_out/golden_r2b.log 2>&1 || { tail -30 gpurun_out/golden_r2b.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_r2b_default.json 2> gpurun_out/bench_r2b_default.err || { tail -20 gpurun_out/bench_r2b_default.err; exit 1; }
cat gpurun_out/bench_r2b_default.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 1 > gpurun_out/bench_r2b_latency.json 2> gpurun_out/bench_r2b_latency.err || { tail -20 gpurun_out/bench_r2b_latency.err; exit 1; }
cat gpurun_out/bench_r2b_latency.json
