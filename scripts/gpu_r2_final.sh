#!/bin/bash
# round 2 final: full GPU tests (goldens included), smoke, K2 solo latency with its family table,
# default SD1.5 bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
timeout -k 10 600 python bench.py --model kandinsky2 --steps 3 --warmup 1 --concurrent 1 --group 1 > $O/bench_k2_latency.json 2> $O/bench_k2_latency.err || { tail -20 $O/bench_k2_latency.err; exit 1; }
cat $O/bench_k2_latency.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_sd_default.json 2> $O/bench_sd_default.err || { tail -20 $O/bench_sd_default.err; exit 1; }
cat $O/bench_sd_default.json
