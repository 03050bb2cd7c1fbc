#!/bin/bash
# Staggered two-group conv tiles + the no-early-exit ring loops: bitwise family tests, a per-cfg
# sweep of the hot SD1.5 conv shapes, and an in-process A/B against the previous library build.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-stag}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "all_tile_configs or families_bitwise or folded_layer_norm or geglu or xreg or big_tiles" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -B5 -A30 "^E " $O/tests.log | head -60; exit $rc; fi
step sweep
LAB_CFGS=${LAB_CFGS:-21,22,29,31,32,36,37,38,39} timeout -k 10 500 python -u scripts/conv_lab.py sweep ${SHAPES:-l0_320,l0_640,l0_960,l1_640,l1_1280,l1_1920,l2_1280,l2_2560} > $O/sweep.jsonl 2>$O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cut -c1-400 $O/sweep.jsonl
step libs_ab
timeout -k 10 300 python -u scripts/conv_lab.py libs_ab > $O/ab.jsonl 2>$O/ab.err || { tail -20 $O/ab.err; exit 1; }
cat $O/ab.jsonl
step done
