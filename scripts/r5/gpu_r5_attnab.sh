#!/bin/bash
# Softmax row-max / mask VALU trim in the flash kernels (bitwise neutral): attention + golden GPU tests
# on the new build, then the SD default bench alternating base (ARBIUS_KERNEL_LIB=..._base.so) / new.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5attn}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_golden_gpu.py -k "attention or attn or golden or temporal" \
  -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
for i in 1 2; do
  ( export ARBIUS_KERNEL_LIB=libarbius_kernels_base.so; one sd_base$i --steps 4 --warmup 1 ) || exit 1
  one sd_new$i --steps 4 --warmup 1 || exit 1
done
( export ARBIUS_KERNEL_LIB=libarbius_kernels_base.so; one sdsolo_base --concurrent 1 --group 1 --steps 6 --warmup 2 ) || exit 1
one sdsolo_new --concurrent 1 --group 1 --steps 6 --warmup 2 || exit 1
