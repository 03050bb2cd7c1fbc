#!/bin/bash
# K2 latency mode (split CFG rows on two hardware queues): bitwise test + solo A/B; then the RVM
# blocking-sync A/B, K2 ATen call sites and a 1-stream K2 kernel summary (scripts/r5/gpu_r5_rvmblk.sh).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5k2}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -k "split_cfg" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in off on off on; do
  if [ $v = on ]; then export ARB_K2_SPLIT_CFG=1; else unset ARB_K2_SPLIT_CFG; fi
  timeout -k 10 300 python3 bench.py --model kandinsky2 --concurrent 1 --group 1 --steps 6 --warmup 1 > $O/solo_$v.log 2> $O/solo_$v.err || { tail -20 $O/solo_$v.err; exit 1; }
  echo "k2 solo split=$v $(tail -1 $O/solo_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_task_latency_ms"], d["stage_s"])')"
done
unset ARB_K2_SPLIT_CFG
bash scripts/r5/gpu_r5_rvmblk.sh ${1:-r5k2}
