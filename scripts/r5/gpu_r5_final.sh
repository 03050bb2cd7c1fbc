#!/bin/bash
# Final-tree check of round 5: GPU tests, smoke, driver-default bench and an SD 1-stream kernel summary
# (scripts/gpu_check.sh), then the K2 solo / 4x4 lines and a K2 solo kernel summary (rocprofv3).
set -o pipefail
TAG=${1:-final5}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
bash scripts/gpu_check.sh $TAG || exit 1
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$n'", d["value"], "ms/step", d["ms_per_step"], "p50", d["p50_task_latency_ms"], d.get("stage_s"))'
}
run k2_solo --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 || exit 1
run k2 --model kandinsky2 --steps 3 --warmup 1 || exit 1
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/k2prof -o run -- python3 $R/bench.py --model kandinsky2 \
  --concurrent 1 --group 1 --steps 2 --warmup 1 > $O/k2prof.log 2>&1) || { tail -20 $O/k2prof.log; exit 1; }
python scripts/prof_summary.py $O/k2prof/run_results.db --top 45 --md $O/rocprof_k2_solo.md > /dev/null 2>&1; rm -rf $O/k2prof
head -3 $O/rocprof_k2_solo.md
echo done
