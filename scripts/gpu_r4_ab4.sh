#!/bin/bash
# A/B call 4: buffer-resource LDS-DMA (glds + stag2) tests and same-process A/B, the default bench,
# and the VAE-graph stall with per-replay host timing (ARB_GRAPH_DEBUG=1).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab4}
mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== dma buf A/B $(date +%T)"
timeout -k 10 400 python -u scripts/dma_buf_ab.py --rounds 5 > $O/dma_buf_ab.jsonl 2>$O/dma_buf_ab.err || { tail -20 $O/dma_buf_ab.err; exit 1; }
cut -c1-220 $O/dma_buf_ab.jsonl
for v in 1 0 1 0; do
  echo "== bench ARB_DMA_BUF=$v $(date +%T)"
  ARB_DMA_BUF=$v timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/bench_buf$v.log 2>$O/bench_buf$v.err || { tail -20 $O/bench_buf$v.err; exit 1; }
  tail -1 $O/bench_buf$v.log | cut -c1-150
done
for spec in "4 8" "3 8"; do
  set -- $spec
  echo "== bench c$1 g$2 (group-of-8 families) $(date +%T)"
  timeout -k 10 400 python bench.py --steps 4 --warmup 2 --concurrent $1 --group $2 > $O/bench_c$1g$2.log 2>$O/bench_c$1g$2.err \
    || { tail -20 $O/bench_c$1g$2.err; exit 1; }
  tail -1 $O/bench_c$1g$2.log | cut -c1-150
done
echo "== vae graph debug $(date +%T)"
ARB_VAE_GRAPH=1 ARB_GRAPH_DEBUG=1 timeout -k 10 400 python bench.py --steps 4 --warmup 2 --concurrent 2 > $O/vg_dbg.log 2>$O/vg_dbg.err \
  || { tail -20 $O/vg_dbg.err; exit 1; }
tail -1 $O/vg_dbg.log | cut -c1-150
grep -c "replay" $O/vg_dbg.err; grep "capture\|replay" $O/vg_dbg.err | tail -30 | cut -c1-200
echo "== done $(date +%T)"
