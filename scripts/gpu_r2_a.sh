#!/bin/bash
# round 2 / call A: pin golden CIDs + boot self-test CIDs, then one PMC pass over the SD1.5 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/pin_goldens.py --out gpurun_out/golden_r2a.json --selftest > gpurun_out/golden_r2a.log 2>&1 || { tail -30 gpurun_out/golden_r2a.log; exit 1; }
tail -3 gpurun_out/golden_r2a.log
STEPS=6 bash scripts/gpu_pmc_bench.sh pmc_r2a
