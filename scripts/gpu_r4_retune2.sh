#!/bin/bash
# Family re-tune on the buffer-DMA kernels (bitwise neutral): SD1.5 batch 8 at 4 streams, Kandinsky2
# batch 8 at 2 streams and batch 2 solo; then same-box bench A/Bs of the new table (ARB_CONV_FAMILY).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-rt2}
mkdir -p $O
export TMPDIR=/tmp
F=arbius_amd/ops/csrc/conv_family.inc
TF="timeout -k 10 700 python -u scripts/tune_family.py"
echo "== fam sd8 c4 $(date +%T)"
$TF $O/f1.inc --batch 8 --conc 4 --models sd15 --merge $F > $O/f1.log 2>&1 || { tail $O/f1.log; exit 1; }
grep -c "re-tuned" $O/f1.log
echo "== fam k2 8 c2 $(date +%T)"
$TF $O/f2.inc --batch 8 --conc 2 --models kandinsky2 --res 768 --merge $O/f1.inc > $O/f2.log 2>&1 || { tail $O/f2.log; exit 1; }
grep -c "re-tuned" $O/f2.log
echo "== fam k2 2 $(date +%T)"
$TF $O/f3.inc --batch 2 --models kandinsky2 --res 768 --merge $O/f2.inc > $O/f3.log 2>&1 || { tail $O/f3.log; exit 1; }
grep -c "re-tuned" $O/f3.log
cp $O/f3.inc $O/conv_family.inc
run() {
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | cut -c1-130)"
}
for v in base tuned base tuned; do
  if [ $v = tuned ]; then export ARB_CONV_FAMILY=$O/conv_family.inc; else unset ARB_CONV_FAMILY; fi
  run sd_$v --steps 6 --warmup 2
  run k2_$v --model kandinsky2 --steps 4 --warmup 1
  run k2solo_$v --model kandinsky2 --steps 3 --warmup 1 --concurrent 1 --group 1
done
echo "== done $(date +%T)"
