#!/bin/bash
# Autotune the UNet3D (zeroscope) linear shapes onto the implicit-GEMM kernel, merged into the pinned
# plan table; prints each shape's best vs hipBLASLt.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-tunevid}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/autotune_conv.py $O --models video --gemms-only --merge arbius_amd/ops/csrc/conv_plans.inc > $O/autotune.log 2>&1 || { tail -20 $O/autotune.log; exit 1; }
grep -c MNK $O/autotune.log
echo done
