#!/bin/bash
# Zeroscope plans: tile configs re-timed on the cold-weight microbench at each launch's pinned split (2 concurrent
# copies = the deployed 2 task streams; bitwise-neutral candidates), then a same-box zeroscope A/B with the
# candidate plan override (ARB_CONV_PLANS).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-zsfam}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u scripts/split_study.py --model zeroscopev2xl --max-m 10000000 --only group --keep-split \
  --cold --conc 2 --out $O/zs.jsonl > $O/study.log 2>&1 || { tail -5 $O/study.log; exit 1; }
python3 scripts/split_plan.py $O/zs.jsonl --out $O/zs --keep-splits --solo-step-us 1e12 --group-step-us 1000 | tail -2
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --model zeroscopev2xl "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
cand() { ( export ARB_CONV_PLANS=$O/zs_plans.txt; one "$@" ); }
for i in 1 2; do
  one base$i --steps 2 --warmup 1 || exit 1
  cand cand$i --steps 2 --warmup 1 || exit 1
done
