#!/bin/bash
# RVM: GPU 4:2:0 conversion on the solve path (default) vs RGB download + host conversion
# (ARB_RVM_GPU_YUV=0): bitwise tests, then an interleaved bench A/B; then the K2 ATen call sites.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5yuv}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
timeout -k 10 300 python -u -m pytest tests/test_rvm_gpu.py tests/test_models_gpu.py -k "yuv or rvm" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in rgb yuv rgb yuv; do
  if [ $v = rgb ]; then export ARB_RVM_GPU_YUV=0; else unset ARB_RVM_GPU_YUV; fi
  timeout -k 10 300 python3 bench.py --model robust_video_matting --steps 6 --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "rvm $v $(tail -1 $O/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], "cpu_s/task", r["host_cpu_s_per_task"], "cores", r["host_cores_busy"], d["stage_s"])')"
done
unset ARB_RVM_GPU_YUV
timeout -k 10 300 python -u scripts/aten_gpu_sites.py kandinsky2 --steps 20 > $O/aten_sites_k2.jsonl 2> $O/aten_sites_k2.err || { tail -20 $O/aten_sites_k2.err; exit 1; }
head -14 $O/aten_sites_k2.jsonl | cut -c1-230
