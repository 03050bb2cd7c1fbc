#!/bin/bash
# Re-tune pinned conv plans for the given model families (register-staged cfgs), rebuild, bench.
set -o pipefail
TAG=${1:-retune}
MODELS=${2:-sd15}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python scripts/autotune_conv.py $O --models $MODELS ${AT_FLAGS---legacy-only} --merge arbius_amd/ops/csrc/conv_plans.inc > $O/autotune.log 2>&1 || { tail -20 $O/autotune.log; exit 1; }
tail -3 $O/autotune.log
cp $O/conv_plans.inc arbius_amd/ops/csrc/conv_plans.inc && python -m arbius_amd.ops.build > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for c in ${BENCH_CS:-1 2}; do
  timeout -k 10 300 python bench.py --concurrent $c > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  echo "c$c $(tail -1 $O/bench_c$c.log | cut -c1-130)"
done
