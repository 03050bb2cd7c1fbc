#!/bin/bash
# Re-pin after a numerics change + SD bench + a short zeroscope profile.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pin2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_golden_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u scripts/pin_goldens.py --out $O/golden_cids.json --selftest > $O/pin.log 2>&1 || { tail -20 $O/pin.log; exit 1; }
echo pinned
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_sd.log 2>&1 || { tail -20 $O/bench_sd.log; exit 1; }
tail -1 $O/bench_sd.log | cut -c1-200
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/p_zs -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model zeroscopev2xl --steps 1 --warmup 1 --concurrent 1 --denoise-steps 10 > $O/prof_zs.log 2>&1) || { grep -v "^    @" $O/prof_zs.log | tail -20; exit 1; }
python scripts/prof_summary.py $O/p_zs/run_results.db --top 40 --md $O/rocprof_zeroscope.md > /dev/null 2>&1; rm -rf $O/p_zs
head -30 $O/rocprof_zeroscope.md | cut -c1-150
echo done
