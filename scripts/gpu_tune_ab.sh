#!/bin/bash
# Kernel tests -> autotune (AT_FLAGS) -> rebuild with the new table -> A/B bench, old table (loaded
# at run time via ARB_CONV_PLANS) vs new, on the same box.
set -o pipefail
TAG=${1:-tuneab}
MODELS=${2:-sd15}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYK:-conv or gemm or tile or persistent}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp arbius_amd/ops/csrc/conv_plans.inc $O/plans_old.inc
timeout -k 10 900 python scripts/autotune_conv.py $O --models $MODELS ${AT_FLAGS:---mode glds --batch 8} --merge arbius_amd/ops/csrc/conv_plans.inc > $O/autotune.log 2>&1 || { tail -20 $O/autotune.log; exit 1; }
cp $O/conv_plans.inc arbius_amd/ops/csrc/conv_plans.inc && python -m arbius_amd.ops.build > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for r in 1 2; do
  ARB_CONV_PLANS=$O/plans_old.inc timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench_old_$r.log 2>&1 || { tail -20 $O/bench_old_$r.log; exit 1; }
  echo "old$r $(tail -1 $O/bench_old_$r.log | cut -c1-120)"
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench_new_$r.log 2>&1 || { tail -20 $O/bench_new_$r.log; exit 1; }
  echo "new$r $(tail -1 $O/bench_new_$r.log | cut -c1-120)"
done
