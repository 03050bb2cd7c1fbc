#!/bin/bash
# Round 5 batch 1: attention512 (tests + TFLOP/s table), then cfg 45 (conv_stag2 192x192): bitwise
# tests, Kandinsky2 family re-tune at batch 8 under 2 streams (every candidate bitwise against the
# pinned plan), same-box K2 bench A/B of the re-tuned table against the built-in one.
set -o pipefail
O=gpurun_out/${1:-r5b1}; mkdir -p $O
export TMPDIR=/tmp
echo "== a512 tests $(date +%T)"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention512 or large_head" > $O/a512_tests.log 2>&1 || { tail -40 $O/a512_tests.log; exit 1; }
tail -2 $O/a512_tests.log
timeout -k 10 300 python -u scripts/attn512_bench.py --json $O/attn512.jsonl > $O/a512_bench.log 2>&1 || { tail -20 $O/a512_bench.log; exit 1; }
cat $O/attn512.jsonl
echo "== cfg45 tests $(date +%T)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "45 or stag2 or lds_dma or family or split" > $O/c45_tests.log 2>&1 || { tail -30 $O/c45_tests.log; exit 1; }
tail -1 $O/c45_tests.log
echo "== k2 tune $(date +%T)"
timeout -k 10 800 python -u scripts/tune_family.py $O/f.inc --batch 8 --conc 2 --models kandinsky2 --res 768 --merge arbius_amd/ops/csrc/conv_family.inc > $O/tune.log 2>&1 || { tail $O/tune.log; exit 1; }
grep -E "re-tuned|-> cfg 45" $O/tune.log | head -20
i=0
for v in base tuned base tuned; do
  i=$((i+1))
  if [ $v = tuned ]; then export ARB_CONV_FAMILY=$O/f.inc; else unset ARB_CONV_FAMILY; fi
  timeout -k 10 400 python bench.py --model kandinsky2 --steps 4 --warmup 1 > $O/k2_${v}_$i.log 2>$O/k2_${v}_$i.err || { tail -20 $O/k2_${v}_$i.err; exit 1; }
  echo "$v $(tail -1 $O/k2_${v}_$i.log | cut -c1-110)"
done
echo "== done $(date +%T)"
