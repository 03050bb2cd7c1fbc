#!/bin/bash
# GPU round trip without rebuilding (the in-tree .so files travel with the snapshot):
# kernel/model tests -> smoke -> 1-GPU bench (driver defaults) -> rocprofv3 kernel stats.
set -o pipefail
TAG=${1:-chk}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -B5 -A30 "^E " $O/pytest_gpu.log | head -80; exit $rc; fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
if [ "${SKIP_PROF:-0}" != "1" ]; then
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 1 --warmup 1 --concurrent 1 > $O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
  python scripts/prof_summary.py $O/prof/run_results.db --top 50 --md $O/rocprof.md > /dev/null 2>&1; rm -rf $O/prof
fi
echo done
