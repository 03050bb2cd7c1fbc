#!/bin/bash
# A/B of two in-tree kernel-library builds (ARBIUS_KERNEL_LIB): kernel tests on B, attention
# microbench and SD1.5 bench on both.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-lib_ab}
B=${LIB_B:-libarbius_kernels_b.so}
mkdir -p $O
ARBIUS_KERNEL_LIB=$B timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-attention or attn}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for l in libarbius_kernels.so $B; do
  ARBIUS_KERNEL_LIB=$l timeout -k 10 300 python scripts/microbench.py $O/micro_$l.json > $O/micro_$l.log 2>&1 || { echo "micro FAIL $l"; tail -20 $O/micro_$l.log; exit 1; }
  python -c "import json; [print('$l', r['op'], r['shape'], r['ours_us']) for r in json.load(open('$O/micro_$l.json')) if r['op'] in '${MICRO_OPS:-attention}'.split(',')]"
done
for rep in 1 2; do for l in libarbius_kernels.so $B; do
  ARBIUS_KERNEL_LIB=$l timeout -k 10 400 python bench.py --steps 4 --warmup 1 ${BENCH_ARGS:-} > $O/bench_$l.$rep.log 2>&1 || { echo "bench FAIL $l"; tail -20 $O/bench_$l.$rep.log; exit 1; }
  echo "$l -> $(tail -1 $O/bench_$l.$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_task_latency_ms"])')"
done; done
