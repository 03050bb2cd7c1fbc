#!/bin/bash
# round 2: (a) re-pin goldens after the CAVLC intra codec (NUMERICS r2.6), RVM / zeroscope bench lines;
# (b) X-in-registers conv tiles (cfg 32-35): GPU tests, then the conv lab sweep against cfg 15 / 21
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2x}
mkdir -p $O
export TMPDIR=/tmp
nproc > $O/nproc.txt
timeout -k 10 900 python -u scripts/pin_goldens.py --out $O/golden.json > $O/golden.log 2>&1 || { tail -30 $O/golden.log; exit 1; }
tail -4 $O/golden.log
timeout -k 10 600 python bench.py --model robust_video_matting --steps 3 --warmup 1 > $O/bench_rvm.json 2> $O/bench_rvm.err || { tail -20 $O/bench_rvm.err; exit 1; }
cat $O/bench_rvm.json
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "xreg or all_tile_configs or geglu" > $O/xreg_tests.txt 2>&1 || { tail -30 $O/xreg_tests.txt; exit 1; }
tail -3 $O/xreg_tests.txt
LAB_CFGS=15,21,32,33,34,35 timeout -k 10 400 python -u scripts/conv_lab.py sweep l0_320,l0_640,l0_960,l1_640,l1_1280,s0_320 > $O/conv_lab_xreg.jsonl 2> $O/conv_lab_xreg.err || { tail -20 $O/conv_lab_xreg.err; exit 1; }
cat $O/conv_lab_xreg.jsonl
timeout -k 10 600 python bench.py --model zeroscopev2xl --steps 3 --warmup 1 > $O/bench_zeroscope.json 2> $O/bench_zeroscope.err || { tail -20 $O/bench_zeroscope.err; exit 1; }
cat $O/bench_zeroscope.json
