#!/bin/bash
# round 2: PMC passes (each its own run: --pmc with --kernel-trace only) on the SD level-0 3x3 conv at
# lock-step batch 8: the X-in-registers tile (cfg 32, planned) against the register-staged 160x128 (cfg 15)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r2pmc}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for cfg in 32 15; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc1_$cfg -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/conv_lab.py pmc l0_320 $cfg > $O/pmc1_$cfg.log 2>&1 || { tail -5 $O/pmc1_$cfg.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc2_$cfg -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/conv_lab.py pmc l0_320 $cfg > $O/pmc2_$cfg.log 2>&1 || { tail -5 $O/pmc2_$cfg.log; exit 1; }
done
ls $O
echo pmc done
