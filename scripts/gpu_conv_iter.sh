#!/bin/bash
# Conv iteration loop: conv kernel tests -> microbench -> SD1.5 bench c1 (+c2).
set -o pipefail
TAG=${1:-conv}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or gemm or splitk or prologue" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/microbench.py > $O/microbench.log 2>&1 || { tail -20 $O/microbench.log; exit 1; }
grep -E "conv3x3|gemm" $O/microbench.log | cut -c1-150
for c in ${CONCS:-1 2}; do
  timeout -k 10 300 python bench.py --concurrent $c > $O/bench_c$c.log 2>&1 || { tail -20 $O/bench_c$c.log; exit 1; }
  echo "c$c $(tail -1 $O/bench_c$c.log | cut -c1-130)"
done
