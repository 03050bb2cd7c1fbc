#!/bin/bash
# Box diagnosis for the round-5 throughput spread (30.5k vs 26k tasks/h on different boxes, same code):
# host CPU share / load, GPU clocks and power, then the default bench with its steady-state kernel
# timeline (are the 4 task streams still 2+-concurrent, or does the GPU idle = host-bound?).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5diag}; mkdir -p $O
export TMPDIR=/tmp
echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') load $(cat /proc/loadavg)"
(rocm-smi --showclocks --showpower --showuse --showtemp 2>&1 | grep -v "^$" | head -30) || true
(cd /tmp && ARB_BENCH_MARKS=1 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 > $O/trace.log 2> $O/trace.err) || { tail -20 $O/trace.err; exit 1; }
grep metric $O/trace.log | cut -c1-120
echo "load after $(cat /proc/loadavg)"
T0=$(grep -o "timed t0 monotonic_ns=[0-9]*" $O/trace.err | grep -o "[0-9]*$")
T1=$(grep -o "timed t1 monotonic_ns=[0-9]*" $O/trace.err | grep -o "[0-9]*$")
python scripts/stream_timeline.py $O/p/run_results.db --window $T0 $T1 --md $O/timeline.md > /dev/null
head -16 $O/timeline.md
python scripts/prof_summary.py $O/p/run_results.db --md $O/rocprof.md > /dev/null 2>&1 || true
rm -rf $O/p
(rocm-smi --showclocks --showpower 2>&1 | grep -v "^$" | head -20) || true
