#!/bin/bash
# attention512: numerics tests (new + the existing d=512 test), then the TFLOP/s table vs the GEMM path.
set -o pipefail
O=gpurun_out/${1:-r5a512}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention512 or large_head" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/attn512_bench.py --json $O/attn512.jsonl > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cat $O/attn512.jsonl
