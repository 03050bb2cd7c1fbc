#!/bin/bash
# One box, one call: K2 per-shape tables + K2 kernel summary, the SD batch-8 table with the pipelined
# attention ring (ARB_ATTN_PP=1) for the A/B against shapes1, then the round-4 check (GPU tests without
# the stale goldens, smoke, default bench, 1x1 norm-prologue A/B).
set -o pipefail
MODELS=kandinsky2 bash scripts/gpu_shapes.sh ${1:-shapes1} \
  && MODELS=anythingv3 LP_GROUPS=4 SKIP_PROF=1 TAGV=_pp EXTRA_ENV=ARB_ATTN_PP=1 bash scripts/gpu_shapes.sh ${1:-shapes1} \
  && bash scripts/gpu_r4_check.sh ${2:-r4chk}
