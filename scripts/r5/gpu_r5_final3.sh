#!/bin/bash
# Last check of the round-5 tree: GPU tests, smoke, driver-default bench, then the SD solo, K2 solo and
# zeroscope lines on the same box.
set -o pipefail
TAG=${1:-final7}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
SKIP_PROF=1 bash scripts/gpu_check.sh $TAG || exit 1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("'$n'", d["value"], "ms/step", d["ms_per_step"], "p50", d["p50_task_latency_ms"], "streams", c.get("streams_per_gpu"), "group", c.get("lockstep_group"))'
}
run sd_solo --concurrent 1 --group 1 --steps 6 --warmup 2 || exit 1
run k2_solo --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 || exit 1
run zs --model zeroscopev2xl --steps 3 --warmup 1 || exit 1
echo done
