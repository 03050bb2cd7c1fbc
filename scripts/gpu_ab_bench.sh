#!/bin/bash
# Kernel tests (PYK filter), then interleaved A/B bench runs: each arg is "ENV=VAL ..." (or "-").
set -o pipefail
TAG=${1:-abb}
shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
if [ -n "${PYK:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "$PYK" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    ev=$e; [ "$ev" = "-" ] && ev=""
    env $ev timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/b_${r}_$i.log 2>&1 || { echo "FAIL $e"; tail -20 $O/b_${r}_$i.log; exit 1; }
    echo "r$r [$e] -> $(tail -1 $O/b_${r}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("p50_task_latency_ms"))')"
  done
done
