#!/bin/bash
# Kandinsky2 diffusion-prior GEMMs (M = 81 tokens x batch, K up to 8192: weight-streaming bound) -
# split-K plan autotune at the canonical batch 8 under 2 streams (moves bytes: re-pin after), the
# solo (batch 2) family re-tune on the new plans, then a same-box K2 bench A/B (2 x 4 and solo)
# of the new tables via ARB_CONV_PLANS / ARB_CONV_FAMILY.
set -o pipefail
TAG=${1:-k2prior}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== plans $(date +%T)"
timeout -k 10 600 python -u scripts/autotune_conv.py $O --models kandinsky2_prior --gemms-only --batch 8 --conc 2 \
  --merge arbius_amd/ops/csrc/conv_plans.inc > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep '"kind"' $O/tune.log | cut -c1-220
echo "== family $(date +%T)"
ARB_CONV_PLANS=$O/conv_plans.inc timeout -k 10 600 python -u scripts/tune_family.py $O/conv_family.inc --batch 2 \
  --models kandinsky2_prior --merge arbius_amd/ops/csrc/conv_family.inc > $O/fam.log 2>&1 || { tail -20 $O/fam.log; exit 1; }
grep "re-tuned" $O/fam.log | head
i=0
for v in base tuned base tuned; do
  i=$((i+1))
  if [ $v = tuned ]; then export ARB_CONV_PLANS=$O/conv_plans.inc ARB_CONV_FAMILY=$O/conv_family.inc
  else unset ARB_CONV_PLANS ARB_CONV_FAMILY; fi
  for m in "2 4" "1 1"; do
    set -- $m
    echo "== k2 $v c$1 g$2 $(date +%T)"
    timeout -k 10 400 python bench.py --model kandinsky2 --steps ${K2_STEPS:-4} --warmup 1 --concurrent $1 --group $2 \
      > $O/k2_${v}_c$1_$i.log 2>$O/k2_${v}_c$1_$i.err || { tail -20 $O/k2_${v}_c$1_$i.err; exit 1; }
    tail -1 $O/k2_${v}_c$1_$i.log | cut -c1-150
  done
done
echo "== done $(date +%T)"
