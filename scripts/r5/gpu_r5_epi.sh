#!/bin/bash
# xreg short-K GEMM epilogue from registers (default build) vs through LDS (lib_ab_epilds.so, built with
# -DARB_XREG_EPI_LDS): bitwise family tests, short-K microbench and the SD bench, same box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5epi}; mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $PT -m gpu tests/test_kernels_gpu.py -k "family or split or geglu or folded or xreg or gemm" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in regs lds; do
  if [ $v = lds ]; then export ARBIUS_KERNEL_LIB=$GRAFT_REPO_ROOT/arbius_amd/ops/lib_ab_epilds.so; else unset ARBIUS_KERNEL_LIB; fi
  timeout -k 10 300 python -u scripts/sk_bench.py --json $O/sk_$v.jsonl > $O/sk_$v.log 2>&1 || { tail -20 $O/sk_$v.log; exit 1; }
  echo "sk $v"; python3 -c "
import json
for l in open('$O/sk_$v.jsonl'):
    d=json.loads(l); print(' ', d['kind'], d['M'], d['N'], d['K'], d['plan'], d['plan_us'], 'us', d['plan_tflops'], 'TF')"
done
for v in lds regs lds regs; do
  if [ $v = lds ]; then export ARBIUS_KERNEL_LIB=$GRAFT_REPO_ROOT/arbius_amd/ops/lib_ab_epilds.so; else unset ARBIUS_KERNEL_LIB; fi
  timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "bench $v $(tail -1 $O/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
done
