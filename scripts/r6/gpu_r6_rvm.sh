#!/bin/bash
# Round 6: RVM with the GPU intra encoder - task streams per GPU (2 / 3 / 4) and the host-encode
# A/B at the default, interleaved, longer runs than gpu_r6_h264.sh (12 steps); host cores per GPU.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6rvm}
mkdir -p $O
export TMPDIR=/tmp
one() {   # name, concurrent, env...
  local n=$1 c=$2; shift 2
  env "$@" timeout -k 10 500 python3 bench.py --model robust_video_matting --concurrent $c --steps 12 --warmup 2 > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; print(d["value"], d["p50_task_latency_ms"], r["host_cpu_s_per_task"], r["host_cores_busy"])')"
}
for rep in a b; do
  one gpu_c2_$rep 2 ARB_RVM_GPU_H264=1 || exit 1
  one gpu_c3_$rep 3 ARB_RVM_GPU_H264=1 || exit 1
  one gpu_c4_$rep 4 ARB_RVM_GPU_H264=1 || exit 1
  one host_c2_$rep 2 ARB_RVM_GPU_H264=0 || exit 1
done
echo "== done $(date +%T)"
