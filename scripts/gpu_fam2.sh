#!/bin/bash
# Bitwise-neutral re-tune pass over every family (incl. the 160-wide staggered tiles): lock-step
# batch-8 (2 streams), solo batch-2 and group-of-2 batch-4 families for SD1.5 + Kandinsky2, and the
# video models' own plans at their pinned splits; rebuild; GPU tests (goldens must not move); bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-fam2}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
TF="timeout -k 10 900 python -u scripts/tune_family.py"
step tests
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "all_tile_configs or families_bitwise" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -A20 "^E " $O/tests.log | head -40; exit $rc; }
F=arbius_amd/ops/csrc/conv_family.inc
step fam8;  $TF $O/f1.inc --batch 8 --conc 2 --models sd15 --merge $F > $O/f1.log 2>&1 || { tail $O/f1.log; exit 1; }
step fam8k; $TF $O/f2.inc --batch 8 --conc 2 --models kandinsky2 --res 768 --merge $O/f1.inc > $O/f2.log 2>&1 || { tail $O/f2.log; exit 1; }
step fam2;  $TF $O/f3.inc --batch 2 --models sd15 --merge $O/f2.inc > $O/f3.log 2>&1 || { tail $O/f3.log; exit 1; }
step fam2k; $TF $O/f4.inc --batch 2 --models kandinsky2 --res 768 --merge $O/f3.inc > $O/f4.log 2>&1 || { tail $O/f4.log; exit 1; }
step fam4;  $TF $O/f5.inc --batch 4 --models sd15 --merge $O/f4.inc > $O/f5.log 2>&1 || { tail $O/f5.log; exit 1; }
step fam4k; $TF $O/fam.inc --batch 4 --models kandinsky2 --res 768 --merge $O/f5.inc > $O/f6.log 2>&1 || { tail $O/f6.log; exit 1; }
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
tail -1 $O/node.log | cut -c1-300
step done
