#!/bin/bash
# round 2: level-0 convs on the X-in-registers / 8-wave tiles (bitwise-neutral re-pin): golden CIDs,
# default SD bench; then the solo-shape tile-family tuning and the latency bench it will be compared to
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2p}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/golden_tests.txt 2>&1 || { tail -30 $O/golden_tests.txt; exit 1; }
tail -2 $O/golden_tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_sd_default.json 2> $O/bench_sd_default.err || { tail -20 $O/bench_sd_default.err; exit 1; }
cat $O/bench_sd_default.json
timeout -k 10 900 python -u scripts/tune_family.py $O/conv_family.inc > $O/tune_family.log 2>&1 || { tail -30 $O/tune_family.log; exit 1; }
grep -c "canonical" $O/tune_family.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 1 > $O/bench_sd_latency.json 2> $O/bench_sd_latency.err || { tail -20 $O/bench_sd_latency.err; exit 1; }
cat $O/bench_sd_latency.json
