#!/bin/bash
# SD1.5 default 3 x 8 (batch-16 families merged) vs the previous 4 x 4: lock-step / golden GPU tests, then
# alternating driver-default benches on one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sdg8ab}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_golden_gpu.py -k "lockstep or golden" -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], c["streams_per_gpu"], c["lockstep_group"])')"
}
for i in 1 2; do
  one c4g4_$i --concurrent 4 --group 4 --steps 3 --warmup 1 || exit 1
  one default_$i || exit 1
done
