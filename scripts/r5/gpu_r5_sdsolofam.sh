#!/bin/bash
# SD1.5 solo (batch 2) tile families on the cold-weight microbench at the pinned splits (bitwise-neutral
# candidates), then the solo latency A/B with the candidate family override, one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sdsolofam}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/split_study.py --model anythingv3 --max-m 100000 --only solo --keep-split --cold \
  --out $O/sd_solo.jsonl > $O/study.log 2>&1 || { tail -5 $O/study.log; exit 1; }
python3 scripts/split_plan.py $O/sd_solo.jsonl --out $O/solo --keep-splits --group-step-us 1e12 | tail -2
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
fam() { ( export ARB_CONV_FAMILY=$O/solo_family.txt; one "$@" ); }
for i in 1 2; do
  one base$i --concurrent 1 --group 1 --steps 6 --warmup 2 || exit 1
  fam fam$i --concurrent 1 --group 1 --steps 6 --warmup 2 || exit 1
done
