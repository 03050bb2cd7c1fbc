#!/bin/bash
# GPU tests + smoke + SD1.5 bench (driver steps) + node / K2 benches + zeroscope at 1 / 2 task streams.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-benches}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
SKIP_PROF=1 BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu_check.sh ${1:-benches} || exit 1
step node
timeout -k 10 400 python bench.py --node --steps 8 --warmup 2 > $O/node.log 2>$O/node.err || { tail -20 $O/node.err; exit 1; }
tail -1 $O/node.log | cut -c1-200
step k2
timeout -k 10 500 python bench.py --model kandinsky2 --steps 4 > $O/k2.log 2>$O/k2.err || { tail -20 $O/k2.err; exit 1; }
tail -1 $O/k2.log | cut -c1-200
for c in 2 1; do
  step zs_c$c
  timeout -k 10 500 python bench.py --model zeroscopev2xl --steps 3 --concurrent $c > $O/zs_c$c.log 2>$O/zs_c$c.err || { tail -20 $O/zs_c$c.err; exit 1; }
  tail -1 $O/zs_c$c.log | cut -c1-200
done
if [ "${PROF:-0}" = "1" ]; then
  step sd_prof_c2
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p_sd -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $O/prof_sd.log 2>&1) || { tail -20 $O/prof_sd.log; exit 1; }
  python scripts/prof_summary.py $O/p_sd/run_results.db --top 50 --md $O/rocprof_sd15_default.md > /dev/null 2>&1; rm -rf $O/p_sd
  head -12 $O/rocprof_sd15_default.md | cut -c1-160
fi
if [ "${PMC:-0}" = "1" ]; then
  step pmc_eager20
  STEPS=20 bash scripts/gpu_pmc_bench.sh ${1:-benches}/pmc || exit 1
fi
step done
