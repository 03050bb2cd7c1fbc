#!/bin/bash
# Round 5 batch 2: attention512 tests + TFLOP/s; family bitwise tests incl. cfg 45 (stag2 192x192) and the
# W-stationary short-K kernel (cfg 46 / 47); short-K microbench; SD GEMM family re-tune restricted to
# {current, 46, 47} under 4 streams + same-box SD A/B; K2 re-tune (all families) + same-box K2 A/B.
set -o pipefail
O=gpurun_out/${1:-r5b2}; mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
echo "== a512 tests $(date +%T)"
timeout -k 10 300 $PT tests/test_kernels_gpu.py -k "attention512 or large_head" > $O/a512_tests.log 2>&1 || { tail -40 $O/a512_tests.log; exit 1; }
tail -1 $O/a512_tests.log
timeout -k 10 300 python -u scripts/attn512_bench.py --json $O/attn512.jsonl > $O/a512_bench.log 2>&1 || { tail -20 $O/a512_bench.log; exit 1; }
cat $O/attn512.jsonl
echo "== family tests $(date +%T)"
timeout -k 10 600 $PT -m gpu tests/test_kernels_gpu.py -k "45 or stag2 or lds_dma or family or split or w_stationary or geglu or folded" > $O/fam_tests.log 2>&1 || { tail -30 $O/fam_tests.log; exit 1; }
tail -1 $O/fam_tests.log
echo "== sk bench $(date +%T)"
timeout -k 10 300 python -u scripts/sk_bench.py --json $O/sk.jsonl > $O/sk.log 2>&1 || { tail -20 $O/sk.log; exit 1; }
cat $O/sk.jsonl
echo "== sd gemm tune $(date +%T)"
timeout -k 10 600 python -u scripts/tune_family.py $O/fsd.inc --batch 8 --conc 4 --models sd15 --gemms-only --families 46,47 --merge arbius_amd/ops/csrc/conv_family.inc > $O/tune_sd.log 2>&1 || { tail $O/tune_sd.log; exit 1; }
grep -E "^gemm|re-tuned" $O/tune_sd.log | head -30
i=0
for v in base tuned base tuned; do
  i=$((i+1))
  if [ $v = tuned ]; then export ARB_CONV_FAMILY=$O/fsd.inc; else unset ARB_CONV_FAMILY; fi
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 > $O/sd_${v}_$i.log 2>$O/sd_${v}_$i.err || { tail -20 $O/sd_${v}_$i.err; exit 1; }
  echo "sd $v $(tail -1 $O/sd_${v}_$i.log | cut -c1-110)"
done
echo "== done $(date +%T)"
