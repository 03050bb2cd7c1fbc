#!/bin/bash
# Same-box A/B of the RVM staging copy (ATen vs numpy), 2 streams, interleaved.  gpurun_out/rvm5/.
set -o pipefail
O=gpurun_out/rvm5; mkdir -p $O
for r in 1 2; do
  for tc in 1 0; do
    ARB_RVM_TORCH_COPY=$tc timeout -k 10 300 python bench.py --model robust_video_matting --steps 6 --warmup 1 > $O/t${tc}_$r.log 2> $O/t${tc}_$r.err || { tail -20 $O/t${tc}_$r.err; exit 1; }
    echo "torch_copy=$tc run$r $(tail -1 $O/t${tc}_$r.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_task_latency_ms"], d["stage_s"])')"
  done
done
