#!/bin/bash
# README lines on the final tree: RVM, SD1.5 / K2 latency mode (1 stream, solo), SD1.5 throughput
# mode (2 streams x groups of 8).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-lines}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
run() { local n=$1; shift; step $n; timeout -k 10 500 python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }; tail -1 $O/$n.log | cut -c1-160; }
run rvm --model robust_video_matting
run sd_latency --concurrent 1 --group 1 --steps 10 --warmup 2
run k2_latency --model kandinsky2 --concurrent 1 --group 1 --steps 4
run sd_c2g8 --group 8 --steps 6 --warmup 2
step done
