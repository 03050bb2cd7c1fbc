#!/bin/bash
# One PMC pass (own run, kernel-trace only) over a short solve without hipGraphs (MODEL, default SD1.5):
# MFMA utilisation and wave-cycle split per kernel (scripts/pmc_summary.py).
set -o pipefail
TAG=${1:-pmc}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/raw -o pmc -- python3 $R/bench.py --model ${MODEL:-anythingv3} --steps 1 --warmup 0 --concurrent 1 --no-graphs --denoise-steps ${STEPS:-6} > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cd $R && python scripts/pmc_summary.py $O/raw --md $O/pmc_summary.md > /dev/null && head -30 $O/pmc_summary.md && rm -rf $O/raw
