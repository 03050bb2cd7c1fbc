#!/bin/bash
# Flash-attention staging A/B: kernel tests, microbench (LDS-DMA on/off), SD1.5 bench (on/off).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-attn_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or attn" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in 0 1; do
  ARB_ATTN_GLDS=$g timeout -k 10 300 python scripts/microbench.py $O/micro_glds$g.json > $O/micro_glds$g.log 2>&1 || { echo "micro FAIL $g"; tail -20 $O/micro_glds$g.log; exit 1; }
  python -c "import json; [print('glds$g', r['shape'], r['ours_us']) for r in json.load(open('$O/micro_glds$g.json')) if r['op']=='attention']"
done
for g in 0 1; do
  ARB_ATTN_GLDS=$g timeout -k 10 400 python bench.py --steps 4 --warmup 1 ${BENCH_ARGS:-} > $O/bench_glds$g.log 2>&1 || { echo "bench FAIL $g"; tail -20 $O/bench_glds$g.log; exit 1; }
  echo "glds$g -> $(tail -1 $O/bench_glds$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_task_latency_ms"])')"
done
