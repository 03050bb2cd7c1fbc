#!/bin/bash
# round 2: solo-shape tile-family table installed: full GPU tests (goldens included), latency and
# default SD bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2f2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 1 > $O/bench_sd_latency.json 2> $O/bench_sd_latency.err || { tail -20 $O/bench_sd_latency.err; exit 1; }
cat $O/bench_sd_latency.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_sd_default.json 2> $O/bench_sd_default.err || { tail -20 $O/bench_sd_default.err; exit 1; }
cat $O/bench_sd_default.json
