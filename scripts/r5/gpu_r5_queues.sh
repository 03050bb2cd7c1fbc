#!/bin/bash
# Round 5, stream -> hardware-queue evidence:
#  1. queue_probe.py: do pool streams / the 4 SD forks' streams overlap a one-CU spin kernel, or run
#     one after another (shared HSA queue)?
#  2. rocprofv3 kernel trace of the default 4-stream SD bench, cut to the timed region
#     (ARB_BENCH_MARKS=1), grouped by HIP stream and by HW queue (scripts/stream_timeline.py).
#  3. the same bench without the profiler (this box's baseline).
set -o pipefail
TAG=${1:-r5q}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== probe pool $(date +%T)"
timeout -k 10 240 python -u scripts/queue_probe.py > $O/probe_pool.jsonl 2> $O/probe_pool.err || { tail -20 $O/probe_pool.err; exit 1; }
cat $O/probe_pool.jsonl
echo "== probe forks $(date +%T)"
timeout -k 10 400 python -u scripts/queue_probe.py --forks 4 > $O/probe_forks.jsonl 2> $O/probe_forks.err || { tail -20 $O/probe_forks.err; exit 1; }
cat $O/probe_forks.jsonl
echo "== trace $(date +%T)"
(cd /tmp && ARB_BENCH_MARKS=1 timeout -k 10 500 rocprofv3 --kernel-trace -d $O/p -o run -- python3 $R/bench.py --steps ${STEPS:-4} --warmup 1 \
   > $O/trace.log 2> $O/trace.err) || { tail -20 $O/trace.err; exit 1; }
grep metric $O/trace.log | cut -c1-160
T0=$(grep -o "timed t0 monotonic_ns=[0-9]*" $O/trace.err | grep -o "[0-9]*$")
T1=$(grep -o "timed t1 monotonic_ns=[0-9]*" $O/trace.err | grep -o "[0-9]*$")
B0=$(grep -o "t0 monotonic_ns=[0-9]* boottime_ns=[0-9]*" $O/trace.err | grep -o "[0-9]*$")
B1=$(grep -o "t1 monotonic_ns=[0-9]* boottime_ns=[0-9]*" $O/trace.err | grep -o "[0-9]*$")
echo "window mono $T0 $T1 boot $B0 $B1"
python scripts/stream_timeline.py $O/p/run_results.db --window $T0 $T1 --md $O/timeline_stream.md > /dev/null
python scripts/stream_timeline.py $O/p/run_results.db --window $T0 $T1 --by queue_id --md $O/timeline_queue.md > /dev/null
python scripts/stream_timeline.py $O/p/run_results.db --window $B0 $B1 --md $O/timeline_stream_boot.md > /dev/null
head -30 $O/timeline_stream.md
head -14 $O/timeline_queue.md
python scripts/prof_summary.py $O/p/run_results.db --md $O/rocprof.md > /dev/null 2>&1 || true
rm -rf $O/p
echo "== bench $(date +%T)"
timeout -k 10 400 python bench.py --steps 8 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.log | cut -c1-200
echo "== done $(date +%T)"
