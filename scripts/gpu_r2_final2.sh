#!/bin/bash
# round 2 final (2): family table with batch-4 entries: full GPU tests (goldens), smoke, groups-of-2 and
# default SD1.5 bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2final2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-120
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 2 > $O/bench_sd_c1g2.json 2> $O/bench_sd_c1g2.err || { tail -20 $O/bench_sd_c1g2.err; exit 1; }
cat $O/bench_sd_c1g2.json
timeout -k 10 300 python bench.py > $O/bench_sd_default.json 2> $O/bench_sd_default.err || { tail -20 $O/bench_sd_default.err; exit 1; }
cat $O/bench_sd_default.json
