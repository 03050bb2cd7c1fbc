#!/bin/bash
# Full GPU tests (goldens deselected), re-pin, then the bench lines of every BASELINE model.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pin4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_golden_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u scripts/pin_goldens.py --out $O/golden_cids.json --selftest > $O/pin.log 2>&1 || { tail -20 $O/pin.log; exit 1; }
echo pinned
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_sd.log 2>&1 || { tail -5 $O/bench_sd.log; exit 1; }
tail -1 $O/bench_sd.log | cut -c1-120
ARBIUS_BENCH_STACKDUMP=60 timeout -k 10 500 python -u bench.py --model zeroscopev2xl --steps 3 --warmup 1 > $O/bench_zs.log 2>&1 || { grep -v "^  File" $O/bench_zs.log | tail -5; exit 1; }
tail -1 $O/bench_zs.log | cut -c1-120
timeout -k 10 500 python -u bench.py --model kandinsky2 --steps 3 --warmup 1 > $O/bench_k2.log 2>&1 || { tail -5 $O/bench_k2.log; exit 1; }
tail -1 $O/bench_k2.log | cut -c1-120
echo done
