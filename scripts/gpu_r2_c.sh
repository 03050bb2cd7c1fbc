#!/bin/bash
# round 2 / call C: autotune the 8-wave 3-stage conv tiles (cfg 28-31) against the pinned plans
set -o pipefail
mkdir -p gpurun_out/tune_r2c
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/autotune_conv.py gpurun_out/tune_r2c --mode deep --batch 8 --conc 2 \
  --merge arbius_amd/ops/csrc/conv_plans.inc > gpurun_out/tune_r2c/log.txt 2>&1 || { tail -30 gpurun_out/tune_r2c/log.txt; exit 1; }
tail -5 gpurun_out/tune_r2c/log.txt
