#!/bin/bash
# Round-4 check on one MI355X: GPU tests (goldens skipped until the re-pin), smoke, default bench,
# and the 1x1 GroupNorm-prologue A/B (ARBIUS_NORM_PROLOGUE=1x1 vs default) on the same box.
set -o pipefail
TAG=${1:-r4chk}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${PYTEST_K:-not golden and not selftest}" > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -B5 -A40 "^E " $O/pytest_gpu.log | head -120; exit $rc; fi
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
for v in ${VARIANTS:-default 1x1 lnfold}; do
  step "bench $v"
  if [ $v = default ]; then
    timeout -k 10 400 python bench.py --steps 12 --warmup 3 > $O/bench_$v.log 2>$O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  elif [ $v = lnfold ]; then
    ARB_LN_FOLD_NARROW=1 timeout -k 10 400 python bench.py --steps 12 --warmup 3 > $O/bench_$v.log 2>$O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  elif [ $v = pp ]; then
    ARB_ATTN_PP=1 timeout -k 10 400 python bench.py --steps 12 --warmup 3 > $O/bench_$v.log 2>$O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  else
    ARBIUS_NORM_PROLOGUE=$v timeout -k 10 400 python bench.py --steps 12 --warmup 3 > $O/bench_$v.log 2>$O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  fi
  tail -1 $O/bench_$v.log | cut -c1-220
done
step done
