#!/bin/bash
# Round-3 sweeps: PMC over the graphed 2-stream SD1.5 bench (20 denoise steps; rocprofv3 serialises
# dispatches under --pmc), zeroscope task streams (1 / 3), SD1.5 stream x group configurations.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-sweep3}
mkdir -p $O/pmc
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tile_tests
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "all_tile_configs or families_bitwise or temb" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -A20 "^E " $O/tests.log | head -40; exit $rc; }
step lab
LAB_CFGS=20,21,23,36,39,40,42,43,44 timeout -k 10 400 python -u scripts/conv_lab.py sweep l0_320,l0_640,l0_960,l1_640,l1_1280,l2_1280 > $O/lab.jsonl 2>$O/lab.err || { tail -20 $O/lab.err; exit 1; }
cut -c1-330 $O/lab.jsonl
step pmc_graphs
(cd /tmp && timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc/raw -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --denoise-steps 20 > $O/pmc/pmc.log 2>&1) || { tail -20 $O/pmc/pmc.log; exit 1; }
python scripts/pmc_summary.py $O/pmc/raw --md $O/pmc/pmc_summary.md > /dev/null && head -3 $O/pmc/pmc_summary.md && rm -rf $O/pmc/raw
for c in 1 3; do
  step zs_c$c
  timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 --concurrent $c > $O/zs_c$c.log 2>$O/zs_c$c.err || { tail -20 $O/zs_c$c.err; exit 1; }
  tail -1 $O/zs_c$c.log | cut -c1-160
done
for cg in "2 6" "2 8" "3 4"; do
  set -- $cg
  step sd_c$1_g$2
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --concurrent $1 --group $2 > $O/sd_c$1_g$2.log 2>$O/sd_c$1_g$2.err || { tail -20 $O/sd_c$1_g$2.err; exit 1; }
  tail -1 $O/sd_c$1_g$2.log | cut -c1-160
done
step done
