#!/bin/bash
# round 2: re-pin goldens after the CAVLC intra codec (NUMERICS r2.6), then RVM / zeroscope bench lines
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2codec}
mkdir -p $O
export TMPDIR=/tmp
nproc > $O/nproc.txt
timeout -k 10 900 python -u scripts/pin_goldens.py --out $O/golden.json > $O/golden.log 2>&1 || { tail -30 $O/golden.log; exit 1; }
tail -4 $O/golden.log
timeout -k 10 600 python bench.py --model robust_video_matting --steps 3 --warmup 1 > $O/bench_rvm.json 2> $O/bench_rvm.err || { tail -20 $O/bench_rvm.err; exit 1; }
cat $O/bench_rvm.json
timeout -k 10 600 python bench.py --model zeroscopev2xl --steps 3 --warmup 1 > $O/bench_zeroscope.json 2> $O/bench_zeroscope.err || { tail -20 $O/bench_zeroscope.err; exit 1; }
cat $O/bench_zeroscope.json
