#!/bin/bash
# round 2 / call D: re-pin goldens (NUMERICS r2.2), SD bench default + latency, rocprof of the default
# bench, and zeroscope / RVM bench lines with their rocprof kernel summaries
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/pin_goldens.py --out $O/golden.json --selftest > $O/golden.log 2>&1 || { tail -30 $O/golden.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_sd_default.json 2> $O/bench_sd_default.err || { tail -20 $O/bench_sd_default.err; exit 1; }
cat $O/bench_sd_default.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 1 > $O/bench_sd_latency.json 2> $O/bench_sd_latency.err || { tail -20 $O/bench_sd_latency.err; exit 1; }
cat $O/bench_sd_latency.json
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/p_sd/run_results.db --top 45 --md $O/rocprof_sd15_default.md > /dev/null && rm -rf $O/p_sd
head -12 $O/rocprof_sd15_default.md | cut -c1-160
timeout -k 10 600 python bench.py --model zeroscopev2xl --steps 3 --warmup 1 > $O/bench_zeroscope.json 2> $O/bench_zeroscope.err || { tail -20 $O/bench_zeroscope.err; exit 1; }
cat $O/bench_zeroscope.json
timeout -k 10 600 python bench.py --model robust_video_matting --steps 3 --warmup 1 > $O/bench_rvm.json 2> $O/bench_rvm.err || { tail -20 $O/bench_rvm.err; exit 1; }
cat $O/bench_rvm.json
MODELS="zeroscopev2xl robust_video_matting" bash scripts/gpu_prof_models.sh r2d_models
