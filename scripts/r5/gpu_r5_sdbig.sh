#!/bin/bash
# SD1.5 lock-step groups beyond 8 (the sampler step now runs one launch per 8 tasks): batch 24-32 on the
# batch-8 canonical plans (families untuned) vs the 3 x 8 default, one box; plus the lock-step GPU tests.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sdbig}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py -k "lockstep or sampler" -x -q --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], d.get("peak_hbm_gb"))')"
}
one default --steps 3 --warmup 1 || exit 1
one c2g16 --concurrent 2 --group 16 --steps 2 --warmup 1 || exit 1
one c3g12 --concurrent 3 --group 12 --steps 2 --warmup 1 || exit 1
one c2g12 --concurrent 2 --group 12 --steps 2 --warmup 1 || exit 1
one default_b --steps 3 --warmup 1 || exit 1
