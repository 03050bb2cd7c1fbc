#!/bin/bash
# round 2 last: RVM (2 slots) and zeroscope bench lines on the final tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2last}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --model robust_video_matting --steps 4 --warmup 1 > $O/bench_rvm.json 2> $O/bench_rvm.err || { tail -20 $O/bench_rvm.err; exit 1; }
cat $O/bench_rvm.json
timeout -k 10 600 python bench.py --model zeroscopev2xl --steps 3 --warmup 1 > $O/bench_zeroscope.json 2> $O/bench_zeroscope.err || { tail -20 $O/bench_zeroscope.err; exit 1; }
cat $O/bench_zeroscope.json
