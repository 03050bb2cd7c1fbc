#!/bin/bash
# Round-4 kernel evidence of the deployed SD1.5 configuration: a PMC pass (eager, one stream: MFMA
# utilisation per kernel), a rocprofv3 kernel summary of the default 4-stream bench and its per-stream
# timeline (scripts/stream_timeline.py).
set -o pipefail
TAG=${1:-prof4}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "== pmc $(date +%T)"
bash scripts/gpu_pmc_bench.sh ${TAG}_pmc_sd || exit 1
echo "== rocprof default $(date +%T)"
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
  > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
grep metric $O/prof_sd.log | cut -c1-160
python scripts/prof_summary.py $O/p_sd/run_results.db --top 50 --md $O/rocprof_sd15_default.md > /dev/null 2>&1
python scripts/stream_timeline.py $O/p_sd/run_results.db --md $O/timeline_sd15_default.md | head -14
rm -rf $O/p_sd
head -12 $O/rocprof_sd15_default.md | cut -c1-160
echo "== done $(date +%T)"
