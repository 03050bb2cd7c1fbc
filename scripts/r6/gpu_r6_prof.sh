#!/bin/bash
# Round 6 profiles: temporal attention (2 query tiles per pass) tests + goldens + microbench vs round 5;
# SD per-op table at the deployed lock-step group of 8 (layer_prof, isolated ops) and the rocprofv3 kernel
# summary of the deployed 3 x 8 bench (the mix); K2 solo kernel summary (dispatches per UNet step);
# zeroscope line.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6prof}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "temporal" -q --timeout 300 --timeout-method thread > $O/pytest_ta.log 2>&1 || { tail -30 $O/pytest_ta.log; exit 1; }
tail -1 $O/pytest_ta.log
timeout -k 10 900 python -u -m pytest tests/test_golden_gpu.py -x -q --timeout 600 --timeout-method thread > $O/pytest_golden.log 2>&1 || { tail -40 $O/pytest_golden.log; exit 1; }
tail -1 $O/pytest_golden.log
step temporal_bench
timeout -k 10 300 python scripts/temporal_bench.py --json $O/ta_new.jsonl > $O/ta_new.log 2>&1 || { tail -20 $O/ta_new.log; exit 1; }
grep '^{' $O/ta_new.log
ARBIUS_KERNEL_LIB=lib_r5base.so timeout -k 10 300 python scripts/temporal_bench.py --json $O/ta_base.jsonl > $O/ta_base.log 2>&1 || { tail -20 $O/ta_base.log; exit 1; }
grep '^{' $O/ta_base.log
step layer_prof
timeout -k 10 600 python scripts/layer_prof.py --model anythingv3 --group 8 --steps 2 --md $O/layers_sd_g8.md --json $O/layers_sd_g8.jsonl > $O/layer_prof.log 2>&1 || { tail -20 $O/layer_prof.log; exit 1; }
head -16 $O/layers_sd_g8.md
timeout -k 10 600 python scripts/layer_prof.py --model zeroscopev2xl --steps 2 --md $O/layers_zs.md --json $O/layers_zs.jsonl > $O/layer_prof_zs.log 2>&1 || { tail -20 $O/layer_prof_zs.log; exit 1; }
head -16 $O/layers_zs.md
step rocprof_sd
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/p_sd/run_results.db --top 60 --md $O/rocprof_sd15_3x8.md > /dev/null 2>&1
rm -rf $O/p_sd
head -14 $O/rocprof_sd15_3x8.md | cut -c1-150
step rocprof_k2_solo
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/p_k2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model kandinsky2 --concurrent 1 --group 1 --steps 1 --warmup 1 > $O/prof_k2.log 2>&1) || { tail -20 $O/prof_k2.log; exit 1; }
python scripts/prof_summary.py $O/p_k2/run_results.db --top 40 --md $O/rocprof_k2_solo.md > /dev/null 2>&1; rm -rf $O/p_k2
head -6 $O/rocprof_k2_solo.md | cut -c1-150
step zeroscope
timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 > $O/zs.log 2>&1 || { tail -20 $O/zs.log; exit 1; }
tail -1 $O/zs.log | cut -c1-130
step done
