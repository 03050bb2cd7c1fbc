#!/bin/bash
# Same-box A/B of the round-5 SD throughput regression: blockwise d=512 VAE attention vs the GEMM path
# (ARB_ATTN512=0), graph capture on the fork stream vs a side stream (ARB_CAPTURE_SIDE=1).
set -o pipefail
O=gpurun_out/${1:-r5ab}; mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-default a512off side both default}; do
  unset ARB_ATTN512 ARB_CAPTURE_SIDE
  case $v in a512off) export ARB_ATTN512=0;; side) export ARB_CAPTURE_SIDE=1;; both) export ARB_ATTN512=0 ARB_CAPTURE_SIDE=1;; esac
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "$v $(tail -1 $O/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_s"])')"
done
