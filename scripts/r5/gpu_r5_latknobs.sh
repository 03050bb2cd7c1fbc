#!/bin/bash
# Latency-mode A/B of the launch-count knobs (GroupNorm prologue in the conv operand load, in-launch
# split-K reduction, one-launch GroupNorm stats + table) on the solo K2 and SD tasks, one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5lat}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
one() {   # name, model args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_task_latency_ms"], d.get("stage_s"))')"
}
variant() {   # name, env assignments...
  local n=$1; shift
  ( export "$@"; one k2_$n --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 ) || exit 1
  ( export "$@"; one sd_$n --concurrent 1 --group 1 --steps 6 --warmup 2 ) || exit 1
}
variant base ARB_NOOP=1
variant prologue ARBIUS_NORM_PROLOGUE=1
variant inlaunch ARB_SPLITK_INLAUNCH=1
variant both ARBIUS_NORM_PROLOGUE=1 ARB_SPLITK_INLAUNCH=1
variant gnfused ARB_GN_FUSED=1
variant base2 ARB_NOOP=1
