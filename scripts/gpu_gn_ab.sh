#!/bin/bash
# GroupNorm kernel A/B: norm kernel tests on the default build, then interleaved stats+table timing
# per library in LAB_LIBS.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-gn_ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "norm or group" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u scripts/conv_lab.py gn > $O/gn.log 2>&1 || { tail -20 $O/gn.log; exit 1; }
cat $O/gn.log
