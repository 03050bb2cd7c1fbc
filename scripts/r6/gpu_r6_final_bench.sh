#!/bin/bash
# Round 6 end check, benches: every BASELINE config at the shipped defaults on one box (SD 3 x 8 =
# the driver's default, SD solo, K2 2 x 8, K2 solo, zeroscope, RVM with the GPU encoder).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6final}
mkdir -p $O
export TMPDIR=/tmp
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 600 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], r["host_cores_busy"])')"
}
one sd_default || exit 1
one sd_solo --concurrent 1 --group 1 --steps 8 --warmup 2 || exit 1
one k2_default --model kandinsky2 --steps 3 --warmup 1 || exit 1
one k2_solo --model kandinsky2 --concurrent 1 --group 1 --steps 4 --warmup 1 || exit 1
one zeroscope --model zeroscopev2xl --steps 3 --warmup 1 || exit 1
one rvm --model robust_video_matting --steps 12 --warmup 2 || exit 1
echo "== done $(date +%T)"
