#!/bin/bash
# RVM slot waits: blocking-sync events (default) vs spinning (ARB_RVM_BLOCKING_SYNC=0), interleaved on one
# box; then the K2 ATen call sites (eager solve under torch.profiler).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5blk}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
for v in spin block spin block; do
  if [ $v = spin ]; then export ARB_RVM_BLOCKING_SYNC=0; else unset ARB_RVM_BLOCKING_SYNC; fi
  timeout -k 10 300 python3 bench.py --model robust_video_matting --steps 6 --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "rvm $v $(tail -1 $O/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["per_rank"][0]; print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"], "cpu_s/task", r["host_cpu_s_per_task"], "cores", r["host_cores_busy"])')"
done
unset ARB_RVM_BLOCKING_SYNC
timeout -k 10 400 python -u scripts/aten_gpu_sites.py kandinsky2 --steps 20 > $O/aten_sites_k2.jsonl 2> $O/aten_sites_k2.err || { tail -20 $O/aten_sites_k2.err; exit 1; }
head -16 $O/aten_sites_k2.jsonl | cut -c1-230
# K2 kernel summary at 1 stream (the profiler's queue-intercept fault was only seen with 2-4
# concurrent streams, profiles/graph_serialisation_r5.md §1)
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model kandinsky2 --concurrent 1 --group 1 --steps 2 --warmup 1 > $O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_results.db --top 40 --md $O/rocprof_k2.md > /dev/null 2>&1; rm -rf $O/prof
head -30 $O/rocprof_k2.md | cut -c1-160
