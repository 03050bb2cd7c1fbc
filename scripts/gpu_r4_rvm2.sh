#!/bin/bash
# Encoder A/B on the box CPU (real matting output frames) + RVM bench with / without the
# low-priority encode threads.  Output under gpurun_out/rvm3/.
set -o pipefail
O=gpurun_out/rvm3; mkdir -p $O
Y=tools_bin/rvm_frames.yuv
scripts/h264_ab.sh 4 8 "tools_bin/h264_orig 8 $Y" "tools_bin/h264_head 8 $Y" "tools_bin/h264_cur2 8 $Y" > $O/enc_ab.txt 2>&1; cat $O/enc_ab.txt
for nice in 10 0; do
  ARB_ENCODE_NICE=$nice timeout -k 10 300 python bench.py --model robust_video_matting --steps 6 --warmup 1 --concurrent 2 > $O/c2_n$nice.log 2> $O/c2_n$nice.err || { tail -20 $O/c2_n$nice.err; exit 1; }
  echo "nice$nice $(tail -1 $O/c2_n$nice.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_task_latency_ms"], d["stage_s"])')"
done
ARB_ENCODE_NICE=10 timeout -k 10 300 python bench.py --model robust_video_matting --steps 6 --warmup 1 --concurrent 3 > $O/c3_n10.log 2> $O/c3_n10.err || { tail -20 $O/c3_n10.err; exit 1; }
echo "c3 nice10 $(tail -1 $O/c3_n10.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_task_latency_ms"], d["stage_s"])')"
