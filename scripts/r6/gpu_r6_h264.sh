#!/bin/bash
# Round 6: GPU avc-intra encoder (csrc/h264_intra.hip) - byte equality against the native encoder,
# the RVM solve path on it, the encoder microbench, RVM bench GPU-encode vs host-encode (A/B, host
# cores per clip); zeroscope copy-site attribution (copyBuffer in the PMC pass).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6h264}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ "${DEBUG:-0}" = 1 ]; then
  step debug
  timeout -k 10 300 python scripts/h264_debug.py > $O/h264_debug.log 2>&1 || { tail -30 $O/h264_debug.log; exit 1; }
  cat $O/h264_debug.log
fi
step tests
timeout -k 10 600 python -u -m pytest tests/test_h264_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_h264.log 2>&1 || { tail -40 $O/pytest_h264.log; exit 1; }
tail -1 $O/pytest_h264.log
timeout -k 10 600 python -u -m pytest tests/test_rvm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_rvm.log 2>&1 || { tail -40 $O/pytest_rvm.log; exit 1; }
tail -1 $O/pytest_rvm.log
step h264_bench
timeout -k 10 300 python scripts/h264_bench.py > $O/h264_bench.log 2>&1 || { tail -20 $O/h264_bench.log; exit 1; }
grep '^{' $O/h264_bench.log
step rvm
one() {   # name, env..., bench args via RVMARGS
  local n=$1; shift
  env "$@" timeout -k 10 500 python3 bench.py --model robust_video_matting --steps 6 --warmup 1 > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d.get("per_rank",[{}]); r=r[0] if isinstance(r,list) else r; print(d["value"], d["p50_task_latency_ms"], r.get("host_cpu_s_per_task"), r.get("host_cores_busy"))')"
}
one gpu ARB_RVM_GPU_H264=1 || exit 1
one host ARB_RVM_GPU_H264=0 || exit 1
one gpu_b ARB_RVM_GPU_H264=1 || exit 1
one host_b ARB_RVM_GPU_H264=0 || exit 1
if [ "${ZS:-0}" = 1 ]; then
  step copy_sites_zs
  timeout -k 10 500 python3 scripts/aten_gpu_sites.py zeroscopev2xl --steps 4 > $O/aten_zs.jsonl 2> $O/aten_zs.err || { tail -5 $O/aten_zs.err; exit 1; }
  grep -h copy_op $O/aten_zs.jsonl | head -20
fi
step done
