#!/bin/bash
# One GPU iteration: kernel tests (fp32 oracles), 1-GPU bench at the driver defaults, per-layer profile.
#   bash scripts/gpu_iter.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-iter}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread ${2:+-k "$2"} > $O/kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 $O/kernels.log
if [ $rc -ne 0 ]; then grep -B5 -A30 "^E " $O/kernels.log | head -60; exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.log | cut -c1-300
if [ "${SKIP_LP:-0}" != "1" ]; then
  timeout -k 10 300 python scripts/layer_prof.py --model anythingv3 --group 4 --steps 10 --top 90 > $O/layer_sd15.md 2>$O/layer.err || { tail -5 $O/layer.err; exit 1; }
  head -12 $O/layer_sd15.md
fi
echo done
