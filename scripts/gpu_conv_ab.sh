#!/bin/bash
# Conv kernel-library A/B: conv kernel tests on the default build, then an in-process interleaved
# timing of the planned conv per shape through each library in LAB_LIBS (bitwise cross-check).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-conv_ab}
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or gemm or splitk or prologue" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 600 python -u scripts/conv_lab.py ab ${LAB_SHAPES:-} > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
