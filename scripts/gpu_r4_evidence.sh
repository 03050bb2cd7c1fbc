#!/bin/bash
# Round-4 evidence runs on one MI355X: template-default operating points (zeroscope 1024x576x24,
# anythingv3 / kandinsky2 1024^2: time + peak HBM), zeroscope with >= 6 timed tasks per slot,
# and an RVM slot sweep.  Each bench line lands in gpurun_out/<tag>/<name>.log.
set -o pipefail
TAG=${1:-evid}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {   # name, timeout, bench args...
  local n=$1 to=$2; shift 2
  echo "== $n $(date +%T)"
  timeout -k 10 $to python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | cut -c1-200
}
run zs_1024x576x24 600 --model zeroscopev2xl --res 1024 --height 576 --frames 24 --steps 1 --warmup 1 --concurrent 1
run sd_1024 300 --res 1024 --steps 2 --warmup 1 --concurrent 1 --group 1
run k2_1024 400 --model kandinsky2 --res 1024 --steps 2 --warmup 1 --concurrent 1 --group 1
run zs_576x320_c2 600 --model zeroscopev2xl --steps 6 --warmup 1 --concurrent 2
for c in ${RVM_SLOTS:-2 4 6}; do
  run rvm_c$c 400 --model robust_video_matting --steps 6 --warmup 1 --concurrent $c
done
echo "== done $(date +%T)"
