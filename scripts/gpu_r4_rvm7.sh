#!/bin/bash
# RVM stream sweep after the copy fixes (2 / 3 / 4 streams, then 2 again).  gpurun_out/rvm8/.
set -o pipefail
O=gpurun_out/rvm8; mkdir -p $O
for c in 2 3 4 2; do
  timeout -k 10 300 python bench.py --model robust_video_matting --steps 6 --warmup 1 --concurrent $c > $O/c$c.log 2> $O/c$c.err || { tail -20 $O/c$c.err; exit 1; }
  echo "c$c $(tail -1 $O/c$c.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_task_latency_ms"], d["stage_s"], d["peak_hbm_gb"])')"
done
