#!/bin/bash
# Round-3 model pass on one MI355X: the SD1.5 A/B of the 1x1 GroupNorm prologue, the Kandinsky2 and
# zeroscope benches, and rocprofv3 kernel summaries of SD1.5 (default config) and zeroscope.  One time
# limit per step; the first failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3b}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step sd_prologue_1x1
ARBIUS_NORM_PROLOGUE=1x1 timeout -k 10 300 python bench.py > $O/sd_1x1.log 2>$O/sd_1x1.err || { tail -20 $O/sd_1x1.err; exit 1; }
tail -1 $O/sd_1x1.log | cut -c1-300
step k2_bench
timeout -k 10 400 python bench.py --model kandinsky2 > $O/k2.log 2>$O/k2.err || { tail -20 $O/k2.err; exit 1; }
tail -1 $O/k2.log | cut -c1-700
step zs_bench
timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 > $O/zs.log 2>$O/zs.err || { tail -20 $O/zs.err; exit 1; }
tail -1 $O/zs.log | cut -c1-400
step sd_prof
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/p_sd/run_results.db --top 45 --md $O/rocprof_sd15_default.md > /dev/null 2>&1; rm -rf $O/p_sd
head -40 $O/rocprof_sd15_default.md | cut -c1-160
step zs_prof
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_zs -o run -- python3 $R/bench.py --model zeroscopev2xl --steps 1 --warmup 1 --concurrent 1 > $O/prof_zs.log 2>&1) || { tail -20 $O/prof_zs.log; exit 1; }
python scripts/prof_summary.py $O/p_zs/run_results.db --top 40 --md $O/rocprof_zeroscope.md > /dev/null 2>&1; rm -rf $O/p_zs
head -24 $O/rocprof_zeroscope.md | cut -c1-160
step done
