#!/bin/bash
# Re-pin the gfx950 goldens + boot self-test after a NUMERICS_VERSION bump, then run the GPU tests
# against the fresh pins, the smoke and the default bench, and a rocprofv3 kernel summary of it.
# Copy the pins back here with:  python scripts/pin_goldens.py --apply-from gpurun_out/<tag>/golden_cids.json
set -o pipefail
TAG=${1:-pin}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step pin
timeout -k 10 900 python -u scripts/pin_goldens.py --out $O/golden_cids.json --selftest --apply > $O/pin.log 2>&1 || { tail -30 $O/pin.log; exit 1; }
cat $O/pin.log | cut -c1-200
SKIP_PROF=${SKIP_PROF:-0} bash scripts/gpu_check.sh $TAG
