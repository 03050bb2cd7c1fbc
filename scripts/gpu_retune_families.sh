#!/bin/bash
# Tile tests of the K-half slot tiles, a short lab sweep, then the bitwise-neutral family / plan
# re-tune with every family, rebuild, GPU tests, SD1.5 / node / K2 /
# zeroscope benches and a 20-step eager PMC pass.  First failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-retune}
mkdir -p $O/pmc
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
TF="timeout -k 10 900 python -u scripts/tune_family.py"
step tile_tests
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "all_tile_configs or families_bitwise or temb" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -A20 "^E " $O/tests.log | head -40; exit $rc; }
step lab
LAB_CFGS=20,21,23,36,39,40,42,43,44 timeout -k 10 300 python -u scripts/conv_lab.py sweep l0_320,l0_640,l1_640,l2_1280 > $O/lab.jsonl 2>$O/lab.err || { tail -20 $O/lab.err; exit 1; }
cut -c1-330 $O/lab.jsonl
F=arbius_amd/ops/csrc/conv_family.inc
step fam8;  $TF $O/f1.inc --batch 8 --conc 2 --models sd15 --merge $F > $O/f1.log 2>&1 || { tail $O/f1.log; exit 1; }
step fam8k; $TF $O/f2.inc --batch 8 --conc 2 --models kandinsky2 --res 768 --merge $O/f1.inc > $O/f2.log 2>&1 || { tail $O/f2.log; exit 1; }
step fam2;  $TF $O/f3.inc --batch 2 --models sd15 --merge $O/f2.inc > $O/f3.log 2>&1 || { tail $O/f3.log; exit 1; }
step fam2k; $TF $O/fam.inc --batch 2 --models kandinsky2 --res 768 --merge $O/f3.inc > $O/f4.log 2>&1 || { tail $O/f4.log; exit 1; }
step plans_video; $TF $O/plans.inc --plans --models video --conc 2 > $O/pv.log 2>&1 || { tail $O/pv.log; exit 1; }
step build
cp $O/fam.inc $F && cp $O/plans.inc arbius_amd/ops/csrc/conv_plans.inc && timeout -k 10 600 python -m arbius_amd.ops.build > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
step gputests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E " $O/pytest_gpu.log | head -60; exit $rc; }
step bench_sd
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/sd.log 2>$O/sd.err || { tail -20 $O/sd.err; exit 1; }
tail -1 $O/sd.log | cut -c1-200
step bench_node
timeout -k 10 400 python bench.py --node --steps 8 --warmup 2 > $O/node.log 2>$O/node.err || { tail -20 $O/node.err; exit 1; }
tail -1 $O/node.log | cut -c1-200
step bench_k2
timeout -k 10 500 python bench.py --model kandinsky2 --steps 4 > $O/k2.log 2>$O/k2.err || { tail -20 $O/k2.err; exit 1; }
tail -1 $O/k2.log | cut -c1-200
step bench_zs
timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 > $O/zs.log 2>$O/zs.err || { tail -20 $O/zs.err; exit 1; }
tail -1 $O/zs.log | cut -c1-200
step pmc
STEPS=20 bash scripts/gpu_pmc_bench.sh ${1:-retune}/pmc || exit 1
step done
