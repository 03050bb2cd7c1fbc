#!/bin/bash
# RVM fast path: GPU tests (fp32 oracles), the 2-slot matting bench, and a kernel profile.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-rvm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rvm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -B5 -A30 "^E " $O/tests.log | head -60; exit $rc; fi
timeout -k 10 400 python bench.py --model robust_video_matting > $O/rvm.log 2>$O/rvm.err || { tail -20 $O/rvm.err; exit 1; }
tail -1 $O/rvm.log | cut -c1-500
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model robust_video_matting --steps 1 --warmup 1 --concurrent 1 > $O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_results.db --top 40 --md $O/rocprof_rvm.md > /dev/null 2>&1; rm -rf $O/prof
head -30 $O/rocprof_rvm.md
echo done
