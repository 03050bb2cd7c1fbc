#!/bin/bash
# Bitwise-neutral family re-tune of the lock-step group shapes (batch BATCH, default 8) under CONC concurrent task
# streams (scripts/tune_family.py: every candidate checked bitwise against the pinned plan), then
# a same-box bench A/B of the new table (ARB_CONV_FAMILY: run-time family table, no rebuild)
# against the built-in one, interleaved twice.
set -o pipefail
TAG=${1:-tune}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
F=arbius_amd/ops/csrc/conv_family.inc
TF="timeout -k 10 ${TUNE_TO:-700} python -u scripts/tune_family.py"
echo "== fam_sd $(date +%T)"
$TF $O/f1.inc --batch ${BATCH:-8} --conc ${CONC:-3} --models sd15 --merge $F > $O/f1.log 2>&1 || { tail $O/f1.log; exit 1; }
tail -2 $O/f1.log | cut -c1-200
OUT=$O/f1.inc
if [ -n "$K2" ]; then
  echo "== fam_k2 $(date +%T)"
  $TF $O/f2.inc --batch ${BATCH:-8} --conc ${CONC:-3} --models kandinsky2 --res 768 --merge $O/f1.inc > $O/f2.log 2>&1 || { tail $O/f2.log; exit 1; }
  tail -2 $O/f2.log | cut -c1-200
  OUT=$O/f2.inc
fi
cp $OUT $O/conv_family.inc
i=0
for v in base tuned base tuned; do
  i=$((i+1))
  echo "== bench $v $(date +%T)"
  if [ $v = tuned ]; then export ARB_CONV_FAMILY=$O/conv_family.inc; else unset ARB_CONV_FAMILY; fi
  timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 6 --warmup 2 --concurrent 3 --group 4} > $O/bench_${v}_$i.log 2>$O/bench_${v}_$i.err \
    || { tail -20 $O/bench_${v}_$i.err; exit 1; }
  tail -1 $O/bench_${v}_$i.log | cut -c1-160
done
echo "== done $(date +%T)"
