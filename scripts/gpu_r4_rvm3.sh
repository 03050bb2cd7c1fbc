#!/bin/bash
# RVM GPU tests + 2-stream bench (twice) after the GIL-free staging copy.  gpurun_out/rvm4/.
set -o pipefail
O=gpurun_out/rvm4; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_rvm.py tests/test_golden_gpu.py -k "rvm or matting" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --model robust_video_matting --steps 6 --warmup 1 > $O/c2_$r.log 2> $O/c2_$r.err || { tail -20 $O/c2_$r.err; exit 1; }
  echo "c2 run$r $(tail -1 $O/c2_$r.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_task_latency_ms"], d["stage_s"], d["config"].get("streams_per_gpu"))')"
done
