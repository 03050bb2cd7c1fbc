#!/bin/bash
# Round 6: GPU intra encoder after the analyse-kernel latency work - byte equality, microbench,
# RVM GPU vs host encode (interleaved, 12 steps).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6h264c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_h264_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_h264.log 2>&1 || { tail -40 $O/pytest_h264.log; exit 1; }
tail -1 $O/pytest_h264.log
timeout -k 10 300 python scripts/h264_bench.py > $O/h264_bench.log 2>&1 || { tail -20 $O/h264_bench.log; exit 1; }
grep '^{' $O/h264_bench.log
one() {   # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 500 python3 bench.py --model robust_video_matting --steps 12 --warmup 2 > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; print(d["value"], d["p50_task_latency_ms"], r["host_cpu_s_per_task"], r["host_cores_busy"])')"
}
for rep in a b; do
  one gpu_$rep ARB_RVM_GPU_H264=1 || exit 1
  one host_$rep ARB_RVM_GPU_H264=0 || exit 1
done
echo "== done $(date +%T)"
