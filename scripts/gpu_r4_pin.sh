#!/bin/bash
# Round-4 re-pin after the NUMERICS_VERSION bump (GELU in GEMM epilogues, prescaled-Q attention, GLIDE
# one-pass pool, padded large-head attention): goldens + boot self-test, then every GPU test against
# the fresh pins, the smoke and the default bench (4 streams x groups of 4).
set -o pipefail
SKIP_PROF=1 bash scripts/gpu_pin.sh ${1:-pin4}
