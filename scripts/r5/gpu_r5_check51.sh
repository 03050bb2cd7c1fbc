#!/bin/bash
# Numerics r5.1 check: GPU tests against the fresh pins, smoke, the driver-default bench, then the
# Kandinsky2 solo / 4x4 and SD solo lines (host CPU per task included) on the same box.
set -o pipefail
TAG=${1:-chk51}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
SKIP_PROF=1 bash scripts/gpu_check.sh $TAG || exit 1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; print("'$n'", d["value"], "ms/step", d["ms_per_step"], "p50", d["p50_task_latency_ms"], "cpu_s/task", r["host_cpu_s_per_task"], d.get("stage_s"))'
}
run k2_solo --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 || exit 1
run k2 --model kandinsky2 --steps 4 --warmup 1 || exit 1
run sd_solo --concurrent 1 --group 1 --steps 6 --warmup 2 || exit 1
