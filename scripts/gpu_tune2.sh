#!/bin/bash
# Tests -> autotune conv plans for kandinsky2 + video shapes (merged with the SD table) ->
# rebuild -> benches (sd15 headline, kandinsky2, zeroscope) -> rocprof summaries.
# rocprof databases are summarised on the box and deleted (gpurun_out must stay < 64 MiB).
set -o pipefail
TAG=${1:-t2}
SKIP_TESTS=${SKIP_TESTS:-0}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
python -m arbius_amd.ops.build > $O/build.log 2>&1 || exit 1
if [ "$SKIP_TESTS" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
timeout -k 10 1500 python scripts/autotune_conv.py $O --models kandinsky2,video --legacy-only --merge arbius_amd/ops/csrc/conv_plans.inc > $O/autotune.log 2>&1 || { tail -20 $O/autotune.log; exit 1; }
cp $O/conv_plans.inc arbius_amd/ops/csrc/conv_plans.inc && python -m arbius_amd.ops.build > $O/build2.log 2>&1 || exit 1
prof() {  # prof NAME ARGS...
  local n=$1; shift
  (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run -- python3 $R/bench.py "$@" > $O/prof_$n.log 2>&1) || { tail -30 $O/prof_$n.log; return 1; }
  python scripts/prof_summary.py $O/prof_$n/run_results.db --top 40 --md $O/rocprof_$n.md > /dev/null 2>&1
  rm -rf $O/prof_$n
}
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $O/bench_sd.log 2>&1 || { tail -30 $O/bench_sd.log; exit 1; }
timeout -k 10 600 python bench.py --model kandinsky2 --steps 2 --warmup 1 > $O/bench_k2.log 2>&1 || { tail -30 $O/bench_k2.log; exit 1; }
timeout -k 10 900 python bench.py --model zeroscopev2xl --steps 1 --warmup 1 > $O/bench_zs.log 2>&1 || { tail -30 $O/bench_zs.log; exit 1; }
prof sd --steps 1 --warmup 1 || exit 1
prof k2 --model kandinsky2 --steps 1 --warmup 1 || exit 1
prof zs --model zeroscopev2xl --steps 1 --warmup 0 --denoise-steps 10 || exit 1
tail -1 $O/bench_sd.log; tail -1 $O/bench_k2.log; tail -1 $O/bench_zs.log
echo done
