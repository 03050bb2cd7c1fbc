#!/bin/bash
# SD1.5 lock-step groups of 8 (batch 16 on the batch-8 canonical plans): cold-weight family study of the
# batch-16 launches at the pinned splits (3 concurrent copies; bitwise-neutral candidates), the family
# override it implies (ratio 0 entries), then 4 x 4 (default) vs 3 x 8 / 4 x 8 with and without it.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sdg8}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/split_study.py --model anythingv3 --max-m 100000 --only group --keep-split \
  --cold --conc 3 --group-size 8 --out $O/sd_g8.jsonl > $O/study.log 2>&1 || { tail -5 $O/study.log; exit 1; }
python3 scripts/split_plan.py $O/sd_g8.jsonl --out $O/g8 --keep-splits --solo-step-us 1e12 --group-step-us 1000 | tail -2
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
fam() { ( export ARB_CONV_FAMILY=$O/g8_family.txt; one "$@" ); }
one c4g4 --steps 3 --warmup 1 || exit 1
one c3g8 --concurrent 3 --group 8 --steps 2 --warmup 1 || exit 1
fam c3g8_fam --concurrent 3 --group 8 --steps 2 --warmup 1 || exit 1
fam c4g8_fam --concurrent 4 --group 8 --steps 2 --warmup 1 || exit 1
one c4g4b --steps 3 --warmup 1 || exit 1
fam c3g8_famb --concurrent 3 --group 8 --steps 2 --warmup 1 || exit 1
