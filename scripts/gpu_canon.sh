#!/bin/bash
# Tune plans for the batch-8 (group of 4) SD shapes, rebuild, then A/B the canonical plan batch.
set -o pipefail
TAG=${1:-canon}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python scripts/autotune_conv.py $O --models sd15 --batch 8 --merge arbius_amd/ops/csrc/conv_plans.inc > $O/autotune.log 2>&1 || { tail -20 $O/autotune.log; exit 1; }
cp $O/conv_plans.inc arbius_amd/ops/csrc/conv_plans.inc && python -m arbius_amd.ops.build > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
for canon in 2 8; do
  for cg in "1 1" "2 4"; do
    set -- $cg
    ARBIUS_PLAN_CANON=$canon timeout -k 10 400 python bench.py --concurrent $1 --group $2 > $O/b_k${canon}_c$1_g$2.log 2>&1 || { tail -20 $O/b_k${canon}_c$1_g$2.log; exit 1; }
    echo "canon $canon c$1 g$2: $(tail -1 $O/b_k${canon}_c$1_g$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "p50", d["p50_task_latency_ms"])')"
  done
done
