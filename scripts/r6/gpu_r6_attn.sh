#!/bin/bash
# Round 6 attention: ILP softmax (all query tiles of a key tile at once), gfx950 lane swaps instead of
# ds_bpermute where the registers allow, DMA sources resolved once; temporal attention V^T through LDS
# transposing reads.  All bitwise: attention + golden GPU tests on the new build, the attention microbench
# on the new and the round-5 library (out_sha of a spiked input: same bytes), then the SD driver-default
# bench alternating round-5 library / new library, and one zeroscope line.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6attn3}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -q --timeout 300 --timeout-method thread > $O/pytest_attn.log 2>&1 || { grep -E "^FAILED|passed|failed" $O/pytest_attn.log | head -20; }
tail -1 $O/pytest_attn.log
timeout -k 10 900 python -u -m pytest tests/test_golden_gpu.py -x -q --timeout 600 --timeout-method thread > $O/pytest_golden.log 2>&1 || { tail -40 $O/pytest_golden.log; exit 1; }
tail -1 $O/pytest_golden.log
step microbench
timeout -k 10 400 python scripts/attn_bench.py --json $O/attn_new.jsonl > $O/attn_new.log 2>&1 || { tail -20 $O/attn_new.log; exit 1; }
grep '^{' $O/attn_new.log
ARBIUS_KERNEL_LIB=lib_r5base.so timeout -k 10 400 python scripts/attn_bench.py --json $O/attn_base.jsonl > $O/attn_base.log 2>&1 || { tail -20 $O/attn_base.log; exit 1; }
grep '^{' $O/attn_base.log
for i in 1 2; do
  step sd_base_$i
  ARBIUS_KERNEL_LIB=lib_r5base.so timeout -k 10 300 python bench.py --steps 4 --warmup 1 > $O/sd_base_$i.log 2>&1 || { tail -20 $O/sd_base_$i.log; exit 1; }
  tail -1 $O/sd_base_$i.log | cut -c1-130
  step sd_new_$i
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 > $O/sd_new_$i.log 2>&1 || { tail -20 $O/sd_new_$i.log; exit 1; }
  tail -1 $O/sd_new_$i.log | cut -c1-130
done
step zeroscope
timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 > $O/zs.log 2>&1 || { tail -20 $O/zs.log; exit 1; }
tail -1 $O/zs.log | cut -c1-130
step done
