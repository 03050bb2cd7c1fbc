#!/bin/bash
# Joint-attention A/B (prefix segment vs concatenated K/V on the LDS-DMA kernel), and the zeroscope /
# damo plan-family re-tune on the buffer-DMA kernels (same split-K per shape: bitwise neutral) with a
# same-box zeroscope bench A/B through ARB_CONV_PLANS.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-zst}
mkdir -p $O
export TMPDIR=/tmp
echo "== joint attention A/B $(date +%T)"
timeout -k 10 300 python -u scripts/joint_attn_ab.py > $O/joint_attn_ab.jsonl 2>$O/joint_attn_ab.err || { tail -20 $O/joint_attn_ab.err; exit 1; }
cat $O/joint_attn_ab.jsonl
echo "== plans video c2 $(date +%T)"
timeout -k 10 800 python -u scripts/tune_family.py $O/conv_plans.inc --plans --models video --conc 2 > $O/pv.log 2>&1 || { tail $O/pv.log; exit 1; }
grep -c "cfg" $O/pv.log
for v in base tuned base tuned; do
  if [ $v = tuned ]; then export ARB_CONV_PLANS=$O/conv_plans.inc; else unset ARB_CONV_PLANS; fi
  echo "== zs $v $(date +%T)"
  timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 --warmup 1 > $O/zs_$v.log 2>$O/zs_$v.err || { tail -20 $O/zs_$v.err; exit 1; }
  tail -1 $O/zs_$v.log | cut -c1-140
done
echo "== done $(date +%T)"
