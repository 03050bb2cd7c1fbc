#!/bin/bash
# RVM after the two-phase solve (encode on the slot's tail thread) + encoder SIMD: GPU tests of the
# touched paths, then the 1080p bench at 2 / 3 / 4 streams.  Output under gpurun_out/rvm2/.
set -o pipefail
O=gpurun_out/rvm2; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_rvm.py tests/test_golden_gpu.py tests/test_workers_gpu.py -k "rvm or matting or worker" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 2 3 4; do
  timeout -k 10 300 python bench.py --model robust_video_matting --steps 6 --warmup 1 --concurrent $c > $O/c$c.log 2> $O/c$c.err || { tail -20 $O/c$c.err; exit 1; }
  echo "c$c $(tail -1 $O/c$c.log | cut -c1-400)"
done
