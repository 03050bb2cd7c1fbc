#!/bin/bash
# Kandinsky2 task streams x lock-step group under numerics r5.1 (one box), bracketed by the default.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5k2sweep}; mkdir -p $O
export TMPDIR=/tmp
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --model kandinsky2 "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], d.get("peak_hbm_gb"))')"
}
one c4g4 --steps 3 --warmup 1 || exit 1
one c5g4 --concurrent 5 --group 4 --steps 3 --warmup 1 || exit 1
one c6g4 --concurrent 6 --group 4 --steps 3 --warmup 1 || exit 1
one c4g4b --steps 3 --warmup 1 || exit 1
