#!/bin/bash
# Lock-step group / stream sweep on one MI355X (batch-invariant plans: every group size solves the
# same bytes per task, so this is a pure throughput knob): SD1.5 and Kandinsky2 bench lines.
set -o pipefail
TAG=${1:-groups}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {   # name, bench args...
  local n=$1; shift
  echo "== $n $(date +%T)"
  timeout -k 10 ${TO:-400} python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | cut -c1-160
}
IFS="|" read -ra SDS <<< "${SD_SPECS:-2 6|2 8|3 4}"
for spec in "${SDS[@]}"; do
  set -- $spec
  run sd_c$1_g$2 --steps ${SD_STEPS:-6} --warmup 2 --concurrent $1 --group $2
done
IFS="|" read -ra K2S <<< "${K2_SPECS:-2 4|2 8|1 1}"
for spec in "${K2S[@]}"; do
  set -- $spec
  run k2_c$1_g$2 --model kandinsky2 --steps ${K2_STEPS:-4} --warmup 1 --concurrent $1 --group $2
done
echo "== done $(date +%T)"
