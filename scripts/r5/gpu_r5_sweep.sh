#!/bin/bash
# Streams x lock-step group sweep for Kandinsky2 and zeroscope now that every task stream owns its own
# hardware queue (graphs.task_stream): the r4 sweeps that put K2 at 2 x 4 and zeroscope at 2 streams
# ran with unchecked stream -> queue binding.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5sweep}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; c=d["config"]; print("'$n'", d["value"], "ms/step", d["ms_per_step"], "p50", d["p50_task_latency_ms"], "cores", r["host_cores_busy"], "peak_hbm_gb", d.get("peak_hbm_gb"), d.get("task_stream_queue_check"))'
}
for sg in ${SD_CFGS:-4x4 4x5 4x6 3x6}; do
  s=${sg%x*}; g=${sg#*x}
  run sd_$sg --concurrent $s --group $g --steps ${SD_STEPS:-3} --warmup 1
done
for sg in ${K2_CFGS:-2x4 3x4 4x4 4x2}; do
  s=${sg%x*}; g=${sg#*x}
  run k2_$sg --model kandinsky2 --concurrent $s --group $g --steps ${K2_STEPS:-3} --warmup 1
done
for s in ${ZS_STREAMS:-3}; do
  run zs_c$s --model zeroscopev2xl --concurrent $s --steps 3 --warmup 1
done
