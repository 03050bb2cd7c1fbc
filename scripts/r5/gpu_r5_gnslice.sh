#!/bin/bash
# One-launch small-slice GroupNorm (gn_slice_kernel; numerics change): kernel tests, then same-box A/Bs
# with ARB_GN_SLICE=0 (stats + table + table-apply) vs the default: K2 solo, SD 4x4, K2 4x4, zeroscope.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-gnslice}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "group_norm or norm_table or prologue" -x -q \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
off() { ( export ARB_GN_SLICE=0; one "$@" ); }
off k2solo_off --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 || exit 1
one k2solo_on --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 || exit 1
off sdsolo_off --concurrent 1 --group 1 --steps 6 --warmup 2 || exit 1
one sdsolo_on --concurrent 1 --group 1 --steps 6 --warmup 2 || exit 1
for i in 1 2; do
  off sd_off$i --steps 4 --warmup 1 || exit 1
  one sd_on$i --steps 4 --warmup 1 || exit 1
done
off k2_off --model kandinsky2 --steps 3 --warmup 1 || exit 1
one k2_on --model kandinsky2 --steps 3 --warmup 1 || exit 1
off zs_off --model zeroscopev2xl --steps 2 --warmup 1 || exit 1
one zs_on --model zeroscopev2xl --steps 2 --warmup 1 || exit 1
