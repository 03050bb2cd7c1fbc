#!/bin/bash
# Round 6, Kandinsky2: joint attention (K/V prefix) on the LDS-DMA kernels (bitwise: prefix test + goldens),
# then K2 4 x 4 (round-5 default) vs 3 x 8 with the batch-16 families (merged), K2 solo latency; the
# GPU-copy call sites of K2 and SD (copyBuffer attribution); and the zeroscope PMC pass on this tree.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6k2}
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -q --timeout 300 --timeout-method thread > $O/pytest_attn.log 2>&1 || { grep -E "^FAILED|passed|failed" $O/pytest_attn.log | head; exit 1; }
tail -1 $O/pytest_attn.log
timeout -k 10 900 python -u -m pytest tests/test_golden_gpu.py -x -q --timeout 600 --timeout-method thread > $O/pytest_golden.log 2>&1 || { tail -40 $O/pytest_golden.log; exit 1; }
tail -1 $O/pytest_golden.log
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 500 python3 bench.py --model kandinsky2 "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
step k2
one c4g4 --concurrent 4 --group 4 --steps 3 --warmup 1 || exit 1
one c3g8 --concurrent 3 --group 8 --steps 2 --warmup 1 || exit 1
one c4g4b --concurrent 4 --group 4 --steps 3 --warmup 1 || exit 1
one c3g8b --concurrent 3 --group 8 --steps 2 --warmup 1 || exit 1
one solo --concurrent 1 --group 1 --steps 4 --warmup 1 || exit 1
step copy_sites
timeout -k 10 400 python3 scripts/aten_gpu_sites.py kandinsky2 --steps 10 > $O/aten_k2.jsonl 2> $O/aten_k2.err || { tail -5 $O/aten_k2.err; exit 1; }
timeout -k 10 400 python3 scripts/aten_gpu_sites.py anythingv3 --steps 10 > $O/aten_sd.jsonl 2> $O/aten_sd.err || { tail -5 $O/aten_sd.err; exit 1; }
grep -h copy_op $O/aten_k2.jsonl | head -12
grep -h copy_op $O/aten_sd.jsonl | head -8
step pmc_zs
MODEL=zeroscopev2xl STEPS=2 bash scripts/gpu_pmc_bench.sh ${1:-r6k2}/pmc_zs || exit 1
step done
