#!/bin/bash
# Round-4 A/B call: new-kernel GPU tests (pool / upsample / prescaled attention / padded large-head
# attention), the bitwise-neutral family re-tune at 4 streams with its bench A/B, the prescaled-Q
# attention bench A/B, and the VAE-graph stream traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab2}
mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "pool2 or upsample2 or prescaled or large_head or flash" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "^E " $O/tests.log | head -60; exit $rc; }
for v in ps1 ps0; do
  echo "== bench $v $(date +%T)"
  ARB_ATTN_PRESCALE=${v#ps} timeout -k 10 400 python bench.py --steps 6 --warmup 2 --concurrent 4 --group 4 \
    > $O/bench_$v.log 2>$O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  tail -1 $O/bench_$v.log | cut -c1-160
done
CONC=4 BENCH_ARGS="--steps 6 --warmup 2 --concurrent 4 --group 4" bash scripts/gpu_retune.sh ${2:-tune4} \
  && bash scripts/gpu_graph_trace.sh ${3:-gtrace}
