#!/bin/bash
# Tests -> autotune conv plans for kandinsky2 + video shapes (merged with the SD table) ->
# rebuild -> benches (sd15 headline, kandinsky2, zeroscope) -> rocprof of kandinsky2 and zeroscope.
set -o pipefail
TAG=${1:-t2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -m arbius_amd.ops.build > $O/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
# test failures (rc 1) do not stop the run; a crash / abort / timeout does
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 1500 python scripts/autotune_conv.py $O --models kandinsky2,video --legacy-only --merge arbius_amd/ops/csrc/conv_plans.inc > $O/autotune.log 2>&1 || { tail -20 $O/autotune.log; exit 1; }
cp $O/conv_plans.inc arbius_amd/ops/csrc/conv_plans.inc && python -m arbius_amd.ops.build > $O/build2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/bench_sd.log 2>&1 || { tail -30 $O/bench_sd.log; exit 1; }
timeout -k 10 600 python bench.py --model kandinsky2 --steps 2 --warmup 1 > $O/bench_k2.log 2>&1 || { tail -30 $O/bench_k2.log; exit 1; }
timeout -k 10 900 python bench.py --model zeroscopev2xl --steps 1 --warmup 1 > $O/bench_zs.log 2>&1 || { tail -30 $O/bench_zs.log; exit 1; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_k2 -o run -- python3 $R/bench.py --model kandinsky2 --steps 1 --warmup 1 > $O/prof_k2.log 2>&1 || { tail -30 $O/prof_k2.log; exit 1; }
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof_zs -o run -- python3 $R/bench.py --model zeroscopev2xl --steps 1 --warmup 0 --denoise-steps 10 > $O/prof_zs.log 2>&1 || { tail -30 $O/prof_zs.log; exit 1; }
tail -1 $O/bench_sd.log; tail -1 $O/bench_k2.log; tail -1 $O/bench_zs.log
echo done
