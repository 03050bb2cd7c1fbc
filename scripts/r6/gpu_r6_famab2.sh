#!/bin/bash
# Round 6: five more SD batch-16 GEMM families from scripts/sd_family_sweep.py (bitwise-equal switches) -
# goldens + GEMM family tests, then SD 3 x 8 new vs previous library (lib_pre.so), interleaved x3.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6famab2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_golden_gpu.py -x -q --timeout 600 --timeout-method thread > $O/pytest_golden.log 2>&1 || { tail -30 $O/pytest_golden.log; exit 1; }
tail -1 $O/pytest_golden.log
one() {   # name, lib, bench args...
  local n=$1 lib=$2; shift 2
  ARBIUS_KERNEL_LIB=$lib timeout -k 10 500 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for rep in a b c; do
  one sd_new_$rep libarbius_kernels.so --steps 4 --warmup 1 || exit 1
  one sd_pre_$rep lib_pre.so --steps 4 --warmup 1 || exit 1
done
echo "== done $(date +%T)"
