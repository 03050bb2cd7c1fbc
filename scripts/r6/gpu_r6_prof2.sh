#!/bin/bash
# Round 6: rocprofv3 kernel summaries of the shipped K2 (2 x 8), zeroscope (2 streams) and RVM
# (2 streams, GPU encoder) benches.  Eager (--no-graphs): the profiler's queue intercept crashes on
# hipGraph replays (profiles/graph_serialisation_r5.md).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6prof2}
mkdir -p $O
export TMPDIR=/tmp
prof() {   # name, top, bench args...
  local n=$1 top=$2; shift 2
  echo "== $n $(date +%T)"
  (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/p_$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $O/prof_$n.log 2>&1) || { tail -20 $O/prof_$n.log; exit 1; }
  python scripts/prof_summary.py $O/p_$n/run_results.db --top $top --md $O/rocprof_$n.md > /dev/null 2>&1; rm -rf $O/p_$n
  head -12 $O/rocprof_$n.md | cut -c1-150
}
prof k2_2x8 50 --model kandinsky2 --steps 1 --warmup 1 --no-graphs || exit 1
prof zs 50 --model zeroscopev2xl --steps 1 --warmup 1 --no-graphs || exit 1
prof rvm 40 --model robust_video_matting --steps 6 --warmup 1 || exit 1

echo "== zs_shortk $(date +%T)"
timeout -k 10 600 python3 scripts/zs_shortk.py --json $O/zs_shortk.jsonl > $O/zs_shortk.log 2>&1 || { tail -20 $O/zs_shortk.log; exit 1; }
cut -c1-400 $O/zs_shortk.jsonl
echo "== done2 $(date +%T)"
