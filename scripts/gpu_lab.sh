#!/bin/bash
# GPU health + conv lab: full GPU test suite, conv tile sweep vs hipBLASLt, PMC passes on the
# hottest conv shapes (each pass its own run: --pmc with --kernel-trace only).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-lab}
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 500 python -u scripts/conv_lab.py sweep ${LAB_SHAPES:-} > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
cut -c1-400 $O/sweep.log
cd /tmp
for s in ${PMC_SHAPES:-l0_320 l1_640}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc1_$s -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/conv_lab.py pmc $s > $O/pmc1_$s.log 2>&1 || { tail -5 $O/pmc1_$s.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc2_$s -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/conv_lab.py pmc $s > $O/pmc2_$s.log 2>&1 || { tail -5 $O/pmc2_$s.log; exit 1; }
done
echo lab done
