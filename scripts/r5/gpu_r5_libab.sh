#!/bin/bash
# Same-box A/B of kernel-library builds (ARBIUS_KERNEL_LIB): the pre-round-5 kernels, + the fast GELU,
# and the current tree, on the default SD bench (blockwise d=512 attention off: the older builds lack it).
set -o pipefail
O=gpurun_out/${1:-r5lib}; mkdir -p $O
export TMPDIR=/tmp ARB_ATTN512=0
for v in ${VARIANTS:-old cur gelu old cur}; do
  case $v in old) export ARBIUS_KERNEL_LIB=lib_ab_old.so;; gelu) export ARBIUS_KERNEL_LIB=lib_ab_gelu.so;; cur) unset ARBIUS_KERNEL_LIB;; esac
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "$v $(tail -1 $O/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
