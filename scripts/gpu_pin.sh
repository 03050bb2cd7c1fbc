#!/bin/bash
# After a deliberate numerics change: GPU tests (goldens deselected), re-pin the golden + self-test
# CIDs, then the SD1.5 default bench and short RVM / zeroscope benches.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pin}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_golden_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u scripts/pin_goldens.py --out $O/golden_cids.json --selftest > $O/pin.log 2>&1 || { tail -20 $O/pin.log; exit 1; }
echo pinned
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_sd.log 2>&1 || { tail -20 $O/bench_sd.log; exit 1; }
  tail -1 $O/bench_sd.log | cut -c1-300
  timeout -k 10 400 python -u bench.py --model robust_video_matting --steps 3 --warmup 1 > $O/bench_rvm.log 2>&1 || { tail -20 $O/bench_rvm.log; exit 1; }
  tail -1 $O/bench_rvm.log | cut -c1-300
  timeout -k 10 500 python -u bench.py --model zeroscopev2xl --steps 2 --warmup 1 > $O/bench_zs.log 2>&1 || { tail -20 $O/bench_zs.log; exit 1; }
  tail -1 $O/bench_zs.log | cut -c1-300
fi
echo done
