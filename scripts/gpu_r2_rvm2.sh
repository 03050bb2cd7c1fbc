#!/bin/bash
# round 2: RVM pipeline forks - concurrency bitwise test, then the RVM bench at the default two task slots
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2rvm2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rvm.py tests/test_golden_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 python bench.py --model robust_video_matting --steps 4 --warmup 1 > $O/bench_rvm.json 2> $O/bench_rvm.err || { tail -20 $O/bench_rvm.err; exit 1; }
cat $O/bench_rvm.json
