#!/bin/bash
# Per-shape evidence on one MI355X: layer_prof tables (every conv / GEMM / attention / norm launch
# with shape, tile family, split-K, us and TFLOP/s) for SD1.5 and Kandinsky2 at the lock-step batch
# (group of 4 = batch 8) and solo (batch 2), and a rocprofv3 kernel summary of the 2-stream K2 bench.
# MODELS / LP_GROUPS / SKIP_PROF select a subset; EXTRA_ENV (e.g. ARB_ATTN_PP=1) runs a tagged variant.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-shapes}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
for m in ${MODELS:-anythingv3 kandinsky2}; do
  for g in ${LP_GROUPS:-4 1}; do
    step "layer_prof $m g$g ${TAGV:-}"
    env ${EXTRA_ENV:-ARBIUS_NOP=1} timeout -k 10 300 python scripts/layer_prof.py --model $m --group $g --steps 2 \
      --md $O/shapes_${m}_g$g${TAGV:-}.md --json $O/shapes_${m}_g$g${TAGV:-}.jsonl > $O/lp_${m}_g$g${TAGV:-}.log 2>&1 \
      || { tail -30 $O/lp_${m}_g$g${TAGV:-}.log; exit 1; }
    head -1 $O/shapes_${m}_g$g${TAGV:-}.md | cut -c1-300
  done
done
if [ "${SKIP_PROF:-0}" != "1" ]; then
  step k2_prof
  (cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_k2 -o run -- python3 $R/bench.py --model kandinsky2 --steps 1 --warmup 1 > $O/prof_k2.log 2>&1) || { tail -20 $O/prof_k2.log; exit 1; }
  python scripts/prof_summary.py $O/p_k2/run_results.db --top 50 --md $O/rocprof_k2_default.md > /dev/null 2>&1; rm -rf $O/p_k2
  head -20 $O/rocprof_k2_default.md | cut -c1-160
fi
step done
