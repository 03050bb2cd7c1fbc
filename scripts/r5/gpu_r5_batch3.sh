#!/bin/bash
# Round 5 batch 3: Kandinsky2 family re-tune over every family (incl. cfg 45 stag2 192x192 and the
# W-stationary cfg 46 / 47) at batch 8 under 2 streams, merged onto FAM (default: the built-in table),
# then a same-box K2 bench A/B.
set -o pipefail
O=gpurun_out/${1:-r5b3}; mkdir -p $O
export TMPDIR=/tmp
FAM=${FAM:-arbius_amd/ops/csrc/conv_family.inc}
echo "== k2 aten sites $(date +%T)"
timeout -k 10 300 python -u scripts/aten_gpu_sites.py kandinsky2 --steps 20 > $O/aten_sites.jsonl 2> $O/aten_sites.err || { tail -20 $O/aten_sites.err; exit 1; }
head -12 $O/aten_sites.jsonl | cut -c1-220
echo "== k2 tune $(date +%T)"
timeout -k 10 800 python -u scripts/tune_family.py $O/f.inc --batch 8 --conc 2 --models kandinsky2 --res 768 --merge $FAM ${FAMS:+--families $FAMS} > $O/tune_k2.log 2>&1 || { tail $O/tune_k2.log; exit 1; }
grep -E "re-tuned|-> cfg 4[567]" $O/tune_k2.log | head -20
i=0
for v in base tuned base tuned; do
  i=$((i+1))
  if [ $v = tuned ]; then export ARB_CONV_FAMILY=$O/f.inc; else unset ARB_CONV_FAMILY; fi
  timeout -k 10 400 python bench.py --model kandinsky2 --steps 4 --warmup 1 > $O/k2_${v}_$i.log 2>$O/k2_${v}_$i.err || { tail -20 $O/k2_${v}_$i.err; exit 1; }
  echo "k2 $v $(tail -1 $O/k2_${v}_$i.log | cut -c1-110)"
done
echo "== done $(date +%T)"
