#!/bin/bash
# Final check of the round-4 tree: every GPU test, the smoke, the driver-default bench, and the
# final-tree bench lines (scripts/gpu_r4_final_bench.sh).
set -o pipefail
SKIP_PROF=1 bash scripts/gpu_check.sh ${1:-final} && bash scripts/gpu_r4_final_bench.sh ${2:-fin2}
