#!/bin/bash
# Round-4 bench lines of the final kernels: SD1.5 default (driver-like K/W), Kandinsky2 2 x 4 and solo,
# zeroscope 2 streams (6 timed tasks per slot).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-fin}
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1 to=$2; shift 2
  echo "== $n $(date +%T)"
  timeout -k 10 $to python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | cut -c1-160
}
run sd_default 400 --steps 12 --warmup 3
run k2_c2g4 400 --model kandinsky2 --steps 4 --warmup 1
run k2_solo 300 --model kandinsky2 --steps 4 --warmup 1 --concurrent 1 --group 1
run sd_solo 300 --steps 6 --warmup 2 --concurrent 1 --group 1
run zs_c2 600 --model zeroscopev2xl --steps 6 --warmup 1
run rvm_c2 300 --model robust_video_matting --steps 6 --warmup 1
echo "== done $(date +%T)"
