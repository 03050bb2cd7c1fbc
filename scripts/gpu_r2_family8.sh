#!/bin/bash
# round 2: tile families for the lock-step batch-8 shapes under two concurrent task streams
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2f8}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/tune_family.py $O/conv_family.inc --batch 8 --conc 2 --merge arbius_amd/ops/csrc/conv_family.inc > $O/tune_family8.log 2>&1 || { tail -30 $O/tune_family8.log; exit 1; }
grep -c "canonical" $O/tune_family8.log
