#!/bin/bash
# bench.py sweep over argument sets (each arg one quoted set), one JSON summary line each.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sweep}
shift
mkdir -p $O
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 500 python bench.py $a > $O/s_$i.log 2>&1 || { echo "FAIL $a"; tail -20 $O/s_$i.log; exit 1; }
  echo "[$a] -> $(tail -1 $O/s_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("p50_task_latency_ms"))')"
done
