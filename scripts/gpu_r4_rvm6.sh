#!/bin/bash
# RVM numpy input-copy A/B (interleaved, 2 streams) + the RVM GPU tests.  gpurun_out/rvm7/.
set -o pipefail
O=gpurun_out/rvm7; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_rvm.py tests/test_golden_gpu.py -k "rvm or matting" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for po in 1 0; do
    ARB_RVM_NUMPY_IN=$po timeout -k 10 300 python bench.py --model robust_video_matting --steps 6 --warmup 1 > $O/p${po}_$r.log 2> $O/p${po}_$r.err || { tail -20 $O/p${po}_$r.err; exit 1; }
    echo "numpy_in=$po run$r $(tail -1 $O/p${po}_$r.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_task_latency_ms"], d["stage_s"], d["peak_hbm_gb"])')"
  done
done
