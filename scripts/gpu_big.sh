#!/bin/bash
# 8-wave conv tiles: kernel tests, then re-pin SD1.5 (batch-8 canonical) plans where they win, bench.
set -o pipefail
TAG=${1:-big}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYK:-tile_configs or big_tiles}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AT_FLAGS="${AT_MODE:---big-only} --batch 8" bash scripts/gpu_retune.sh $TAG ${2:-sd15}
