#!/bin/bash
# Round-3 iteration on one MI355X: kernel + RVM GPU tests, the norm-kernel A/B, the RVM and SD1.5
# benches and an RVM kernel profile.  Every GPU step has its own time limit; the first failure ends
# the script (no GPU work after a fault).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py tests/test_rvm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -B5 -A30 "^E " $O/tests.log | head -80; exit $rc; fi
step normbench
ARB_GN_APPLY2=0 ARB_LN_PACKED=0 ARB_GN_FUSED=0 TAG=old timeout -k 10 120 python scripts/norm_bench.py > $O/norm_old.jsonl 2>$O/norm.err || { tail $O/norm.err; exit 1; }
TAG=new timeout -k 10 120 python scripts/norm_bench.py > $O/norm_new.jsonl 2>>$O/norm.err || { tail $O/norm.err; exit 1; }
paste -d' ' <(cut -c1-70 $O/norm_old.jsonl) <(grep -o '"us": [0-9.]*' $O/norm_new.jsonl)
step rvm_bench
timeout -k 10 400 python bench.py --model robust_video_matting > $O/rvm.log 2>$O/rvm.err || { tail -20 $O/rvm.err; exit 1; }
tail -1 $O/rvm.log | cut -c1-600
step rvm_bench_sdma
HSA_ENABLE_SDMA=1 timeout -k 10 400 python bench.py --model robust_video_matting > $O/rvm_sdma.log 2>$O/rvm_sdma.err || { tail -20 $O/rvm_sdma.err; exit 1; }
tail -1 $O/rvm_sdma.log | cut -c1-300
step sd_bench
timeout -k 10 400 python bench.py > $O/sd.log 2>$O/sd.err || { tail -20 $O/sd.err; exit 1; }
tail -1 $O/sd.log | cut -c1-400
step rvm_prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model robust_video_matting --steps 1 --warmup 1 --concurrent 1 > $O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_results.db --top 40 --md $O/rocprof_rvm.md > /dev/null 2>&1; rm -rf $O/prof
head -24 $O/rocprof_rvm.md | cut -c1-200
step done
