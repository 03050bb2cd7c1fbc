#!/bin/bash
# Round 6: SD1.5 streams x lock-step group around the 3 x 8 default with the round-6 kernels.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6sdsweep}
mkdir -p $O
export TMPDIR=/tmp
one() {
  local n=$1; shift
  timeout -k 10 500 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
one c3g8 --concurrent 3 --group 8 --steps 4 --warmup 1 || exit 1
one c4g8 --concurrent 4 --group 8 --steps 3 --warmup 1 || exit 1
one c3g10 --concurrent 3 --group 10 --steps 3 --warmup 1 || exit 1
one c2g12 --concurrent 2 --group 12 --steps 4 --warmup 1 || exit 1
one c4g6 --concurrent 4 --group 6 --steps 4 --warmup 1 || exit 1
one c3g8b --concurrent 3 --group 8 --steps 4 --warmup 1 || exit 1
echo "== done $(date +%T)"
