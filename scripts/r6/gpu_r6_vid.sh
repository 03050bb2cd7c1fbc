#!/bin/bash
# Round 6: zeroscope / damo solve path on the GPU encoder (goldens: byte-identical CIDs), zeroscope
# bench; Kandinsky2 2 x 8 vs 4 x 4 repeated.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6vid}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step goldens
timeout -k 10 900 python -u -m pytest tests/test_golden_gpu.py -x -q --timeout 600 --timeout-method thread > $O/pytest_golden.log 2>&1 || { tail -40 $O/pytest_golden.log; exit 1; }
tail -1 $O/pytest_golden.log
one() {   # name, model, bench args...
  local n=$1 m=$2; shift 2
  timeout -k 10 600 python3 bench.py --model $m "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], r["host_cores_busy"])')"
}
step zeroscope
one zs zeroscopev2xl --steps 2 --warmup 1 || exit 1
step k2
one k2_c2g8 kandinsky2 --concurrent 2 --group 8 --steps 3 --warmup 1 || exit 1
one k2_c4g4 kandinsky2 --concurrent 4 --group 4 --steps 3 --warmup 1 || exit 1
one k2_c2g8b kandinsky2 --concurrent 2 --group 8 --steps 3 --warmup 1 || exit 1
one k2_c4g4b kandinsky2 --concurrent 4 --group 4 --steps 3 --warmup 1 || exit 1
step done
