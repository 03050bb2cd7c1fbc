#!/bin/bash
# Round 6: the GPU intra encoder's first-differing state against its host run, per optimisation level
# of csrc/h264_intra.hip (encoder-only libraries libh264_O{0..3}.so built in-tree).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6h264dbg}
mkdir -p $O
export TMPDIR=/tmp
for o in O0 O1 O2 O3 rowinc; do
  echo "== $o $(date +%T)"
  ARBIUS_KERNEL_LIB=libh264_$o.so timeout -k 10 300 python scripts/h264_debug.py > $O/dbg_$o.log 2>&1 || { tail -20 $O/dbg_$o.log; exit 1; }
  grep -h '"sync": 1' $O/dbg_$o.log | cut -c1-400
  grep -h dbg_diff $O/dbg_$o.log | cut -c1-200
done
