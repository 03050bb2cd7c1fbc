#!/bin/bash
# Task streams on distinct hardware queues (graphs.task_stream) vs the unchecked pool streams, and the
# r4 VAE-graph stall configuration (VAE graph captured on one shared side stream) on the same box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5qf}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
PYTHONFAULTHANDLER=1 timeout -k 10 300 python -u -X faulthandler -m pytest tests/test_queues_gpu.py tests/test_models_gpu.py -k 'queues or vae_graph_two or concurrent_streams' -s -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
val() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], d.get("task_stream_queue_check"))'; }
for v in ${VARIANTS:-check nocheck vae_side vae check}; do
  unset ARB_QUEUE_CHECK ARB_VAE_GRAPH ARB_CAPTURE_SIDE
  case $v in nocheck) export ARB_QUEUE_CHECK=0;; vae_side) export ARB_VAE_GRAPH=1 ARB_CAPTURE_SIDE=1;;
    vae) export ARB_VAE_GRAPH=1;; esac
  timeout -k 10 300 python3 bench.py --steps ${STEPS:-4} --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "$v $(val $O/b_$v.log)"
  grep "task .* done" $O/b_$v.err | tail -8 | tr '\n' ' '; echo
done
