#!/bin/bash
# K2 text/prior linear-routing A/B, then rocprofv3 kernel summaries of the SD1.5 default config and K2.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-fprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/k2_text_ab.py > $O/k2ab.log 2>&1 || { tail -20 $O/k2ab.log; exit 1; }
head -2 $O/k2ab.log
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/p_sd/run_results.db --top 45 --md $O/rocprof_sd15_default.md > /dev/null 2>&1; rm -rf $O/p_sd
head -24 $O/rocprof_sd15_default.md | cut -c1-140
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_k2 -o run -- python3 $R/bench.py --model kandinsky2 --steps 1 --warmup 1 > $O/prof_k2.log 2>&1) || { tail -20 $O/prof_k2.log; exit 1; }
python scripts/prof_summary.py $O/p_k2/run_results.db --top 45 --md $O/rocprof_kandinsky2.md > /dev/null 2>&1; rm -rf $O/p_k2
head -24 $O/rocprof_kandinsky2.md | cut -c1-140
echo done
