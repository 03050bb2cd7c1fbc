#!/bin/bash
# End-to-end A/B of the cold-weight family candidates (scripts/r5/coldfam: same splits, so bitwise neutral):
# SD 4x4, K2 solo and K2 4x4, alternating base / candidate on one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-coldab}; mkdir -p $O
P=$GRAFT_REPO_ROOT/scripts/r5/coldfam
export TMPDIR=/tmp
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
cand() { ( export ARB_CONV_PLANS=$P/plans.txt ARB_CONV_FAMILY=$P/family.txt; one "$@" ); }
for i in 1 2; do
  one sd_base$i --steps 4 --warmup 1 || exit 1
  cand sd_cold$i --steps 4 --warmup 1 || exit 1
done
one k2solo_base --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 || exit 1
cand k2solo_cold --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 || exit 1
one k2_base --model kandinsky2 --steps 3 --warmup 1 || exit 1
cand k2_cold --model kandinsky2 --steps 3 --warmup 1 || exit 1
