#!/bin/bash
# Round-3 evidence pass on one MI355X: zeroscope bench + kernel summary, SD1.5 kernel summary in the
# deployed 2-stream configuration, and a PMC pass (MFMA utilisation per kernel).  One time limit per
# step; the first failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-profiles}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step node_bench
timeout -k 10 400 python bench.py --node --steps 8 --warmup 2 > $O/node.log 2>$O/node.err || { tail -20 $O/node.err; exit 1; }
tail -1 $O/node.log | cut -c1-300
step k2_bench
timeout -k 10 500 python bench.py --model kandinsky2 --steps 4 > $O/k2.log 2>$O/k2.err || { tail -20 $O/k2.err; exit 1; }
tail -1 $O/k2.log | cut -c1-300
step zs_bench
timeout -k 10 600 python bench.py --model zeroscopev2xl --steps 3 > $O/zs.log 2>$O/zs.err || { tail -20 $O/zs.err; exit 1; }
tail -1 $O/zs.log | cut -c1-400
step zs_prof
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_zs -o run -- python3 $R/bench.py --model zeroscopev2xl --steps 1 --warmup 1 --concurrent 1 > $O/prof_zs.log 2>&1) || { tail -20 $O/prof_zs.log; exit 1; }
python scripts/prof_summary.py $O/p_zs/run_results.db --top 40 --md $O/rocprof_zeroscope.md > /dev/null 2>&1; rm -rf $O/p_zs
head -16 $O/rocprof_zeroscope.md | cut -c1-160
step sd_prof_c2
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/p_sd/run_results.db --top 50 --md $O/rocprof_sd15_default.md > /dev/null 2>&1; rm -rf $O/p_sd
head -16 $O/rocprof_sd15_default.md | cut -c1-160
step pmc
bash scripts/gpu_pmc_bench.sh ${1:-profiles}/pmc || exit 1
step done
