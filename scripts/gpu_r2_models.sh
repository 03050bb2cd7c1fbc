#!/bin/bash
# round 2: current-tree bench lines with free-running task slots: SD1.5 default, RVM (2 / 3 slots,
# faster encoder), Kandinsky2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2m}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench_sd_default.json 2> $O/bench_sd_default.err || { tail -20 $O/bench_sd_default.err; exit 1; }
cat $O/bench_sd_default.json
timeout -k 10 600 python bench.py --model robust_video_matting --steps 4 --warmup 1 > $O/bench_rvm_c2.json 2> $O/bench_rvm_c2.err || { tail -20 $O/bench_rvm_c2.err; exit 1; }
cat $O/bench_rvm_c2.json
timeout -k 10 600 python bench.py --model robust_video_matting --steps 4 --warmup 1 --concurrent 3 > $O/bench_rvm_c3.json 2> $O/bench_rvm_c3.err || { tail -20 $O/bench_rvm_c3.err; exit 1; }
cat $O/bench_rvm_c3.json
timeout -k 10 600 python bench.py --model kandinsky2 --steps 3 --warmup 1 > $O/bench_k2.json 2> $O/bench_k2.err || { tail -20 $O/bench_k2.err; exit 1; }
cat $O/bench_k2.json
