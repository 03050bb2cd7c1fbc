#!/bin/bash
# Lock-step group determinism test + bench matrix over (streams, group).
set -o pipefail
TAG=${1:-grp}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lockstep or concurrent_streams" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; [ $rc -ne 0 ] && { grep -B2 -A25 "^E " $O/pytest.log | head -40; exit 1; }
for cg in ${MATRIX:-"1 1" "1 2" "1 4" "2 2" "2 4"}; do
  set -- $cg
  timeout -k 10 400 python bench.py --concurrent $1 --group $2 > $O/bench_c$1_g$2.log 2>&1 || { tail -20 $O/bench_c$1_g$2.log; exit 1; }
  echo "c$1 g$2: $(tail -1 $O/bench_c$1_g$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "p50", d["p50_task_latency_ms"])')"
done
