#!/bin/bash
# Every model's default bench on one box: throughput, latency and the host CPU each task costs
# (bench.py per_rank host_cpu_s_per_task / host_cores_busy) -> profiles/cpu_budget_r5.md.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5models}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg) nproc $(nproc)"
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; c=d["config"]; print("'$n'", d["value"], "ms/step", d["ms_per_step"], "p50", d["p50_task_latency_ms"], "streams", c.get("streams_per_gpu"), "group", c.get("lockstep_group"), "cpu_s/task", r["host_cpu_s_per_task"], "cores", r["host_cores_busy"], d.get("task_stream_queue_check"))'
}
run sd ${SD_ARGS:---steps 6 --warmup 1}
run sd_solo --concurrent 1 --group 1 --steps 6 --warmup 2
run k2 --model kandinsky2 --steps 4 --warmup 1
run k2_solo --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1
run zs --model zeroscopev2xl --steps 4 --warmup 1
run rvm --model robust_video_matting --steps 6 --warmup 1
