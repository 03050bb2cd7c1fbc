#!/bin/bash
# Round 6: Kandinsky2 streams x lock-step group around the 4 x 4 default with the batch-16 families.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6k2sweep}
mkdir -p $O
export TMPDIR=/tmp
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 500 python3 bench.py --model kandinsky2 "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
one c4g4 --concurrent 4 --group 4 --steps 3 --warmup 1 || exit 1
one c4g8 --concurrent 4 --group 8 --steps 2 --warmup 1 || exit 1
one c2g8 --concurrent 2 --group 8 --steps 3 --warmup 1 || exit 1
one c5g4 --concurrent 5 --group 4 --steps 3 --warmup 1 || exit 1
one c3g8 --concurrent 3 --group 8 --steps 2 --warmup 1 || exit 1
one c4g4b --concurrent 4 --group 4 --steps 3 --warmup 1 || exit 1
echo "== done $(date +%T)"
