#!/bin/bash
# A/B of host-side env switches on the SD1.5 bench (1 stream, short): each line "<env> -> json".
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}
mkdir -p $O
shift
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "norm_table_apply or splitk or prologue" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --steps 3 --warmup 1 --concurrent ${CONC:-1} ${BENCH_ARGS:-} > $O/bench_$i.log 2>&1 || { echo "FAIL $e"; tail -20 $O/bench_$i.log; exit 1; }
  echo "$e -> $(tail -1 $O/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_task_latency_ms"], d["stage_s"])')"
done
