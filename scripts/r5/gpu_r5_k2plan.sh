#!/bin/bash
# GroupNorm stats+table tail (bitwise test) and the Kandinsky2 re-plan candidates (scripts/split_study.py
# -> scripts/split_plan.py; ARB_CONV_PLANS / ARB_CONV_FAMILY override files under scripts/r5/k2plans/):
# K2 solo latency, K2 4x4 throughput and the SD default bench per variant, one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5k2plan}; mkdir -p $O
P=$GRAFT_REPO_ROOT/scripts/r5/k2plans
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "group_norm or norm_table" -x -q --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], d.get("stage_s"))')"
}
k2solo() { one k2solo_$1 --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1; }
k2tp() { one k2tp_$1 --model kandinsky2 --steps 3 --warmup 1; }
( export ARB_GN_TAIL=0; k2solo notail ) || exit 1
k2solo tail || exit 1
( export ARB_CONV_PLANS=$P/k2fam_plans.txt ARB_CONV_FAMILY=$P/k2fam_family.txt; k2solo fam ) || exit 1
( export ARB_CONV_PLANS=$P/k2w4800_plans.txt ARB_CONV_FAMILY=$P/k2w4800_family.txt; k2solo w4800 ) || exit 1
( export ARB_CONV_PLANS=$P/k2w1200_plans.txt ARB_CONV_FAMILY=$P/k2w1200_family.txt; k2solo w1200 ) || exit 1
( export ARB_GN_TAIL=0; k2tp notail ) || exit 1
k2tp tail || exit 1
( export ARB_CONV_PLANS=$P/k2fam_plans.txt ARB_CONV_FAMILY=$P/k2fam_family.txt; k2tp fam ) || exit 1
( export ARB_CONV_PLANS=$P/k2w4800_plans.txt ARB_CONV_FAMILY=$P/k2w4800_family.txt; k2tp w4800 ) || exit 1
( export ARB_CONV_PLANS=$P/k2w1200_plans.txt ARB_CONV_FAMILY=$P/k2w1200_family.txt; k2tp w1200 ) || exit 1
( export ARB_GN_TAIL=0; one sd_notail --steps 4 --warmup 1 ) || exit 1
one sd_tail --steps 4 --warmup 1 || exit 1
