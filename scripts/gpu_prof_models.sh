#!/bin/bash
# rocprofv3 kernel stats of one task per model family (Kandinsky2 c1, zeroscope c1).
set -o pipefail
TAG=${1:-profm}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for m in ${MODELS:-kandinsky2 zeroscopev2xl}; do
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/p_$m -o run -- python3 $R/bench.py --model $m --steps 1 --warmup 1 --concurrent 1 > $O/prof_$m.log 2>&1) || { tail -20 $O/prof_$m.log; exit 1; }
  python scripts/prof_summary.py $O/p_$m/run_results.db --top 40 --md $O/rocprof_$m.md > /dev/null 2>&1; rm -rf $O/p_$m
  echo "== $m"; head -14 $O/rocprof_$m.md | cut -c1-150
done
