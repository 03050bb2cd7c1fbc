#!/bin/bash
# GN-prologue fusion milestone: tests -> SD autotune (legacy cfgs, merged) -> benches c1/c2 -> rocprof.
set -o pipefail
TAG=${1:-g1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -m arbius_amd.ops.build > $O/build.log 2>&1 && python -m arbius_amd.native.build >> $O/build.log 2>&1 || exit 1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -B5 -A30 "^E " $O/pytest_gpu.log | head -80; exit $rc; fi
fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --concurrent 1 > $O/bench_sd_c1_pre.log 2>&1 || { tail -20 $O/bench_sd_c1_pre.log; exit 1; }
tail -1 $O/bench_sd_c1_pre.log | cut -c1-220
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_pre -o run -- python3 $R/bench.py --steps 1 --warmup 1 --concurrent 1 > $O/prof_pre.log 2>&1) || { tail -20 $O/prof_pre.log; exit 1; }
python scripts/prof_summary.py $O/prof_pre/run_results.db --top 60 --md $O/rocprof_pre.md > /dev/null 2>&1; rm -rf $O/prof_pre
timeout -k 10 900 python scripts/autotune_conv.py $O --models sd15,kandinsky2,video --legacy-only --merge arbius_amd/ops/csrc/conv_plans.inc > $O/autotune.log 2>&1 || { tail -20 $O/autotune.log; exit 1; }
cp $O/conv_plans.inc arbius_amd/ops/csrc/conv_plans.inc && python -m arbius_amd.ops.build > $O/build2.log 2>&1 || exit 1
for c in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --concurrent $c > $O/bench_sd_c$c.log 2>&1 || { tail -20 $O/bench_sd_c$c.log; exit 1; }
  tail -1 $O/bench_sd_c$c.log | cut -c1-220
done
timeout -k 10 600 python bench.py --model kandinsky2 --steps 2 --warmup 1 --concurrent 2 > $O/bench_k2_c2.log 2>&1 || { tail -20 $O/bench_k2_c2.log; exit 1; }
tail -1 $O/bench_k2_c2.log | cut -c1-220
timeout -k 10 900 python bench.py --model zeroscopev2xl --steps 1 --warmup 1 --concurrent 1 > $O/bench_zs.log 2>&1 || { tail -20 $O/bench_zs.log; exit 1; }
tail -1 $O/bench_zs.log | cut -c1-220
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_sd -o run -- python3 $R/bench.py --steps 1 --warmup 1 --concurrent 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
python scripts/prof_summary.py $O/prof_sd/run_results.db --top 40 --md $O/rocprof_sd.md > /dev/null 2>&1; rm -rf $O/prof_sd
echo done
