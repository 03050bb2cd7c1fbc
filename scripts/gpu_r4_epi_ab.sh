#!/bin/bash
# Epilogue residual-prefetch A/B: the kernel tests on the new build, then per-shape timing and the SD1.5 /
# Kandinsky2 benches against the previous build (ARBIUS_KERNEL_LIB=libarbius_kernels_base.so),
# interleaved on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-epi}
mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in base new; do
  if [ $lib = base ]; then export ARBIUS_KERNEL_LIB=libarbius_kernels_base.so; else unset ARBIUS_KERNEL_LIB; fi
  echo "== shapes $lib $(date +%T)"
  timeout -k 10 400 python -u scripts/dma_buf_ab.py --rounds 3 > $O/shapes_$lib.jsonl 2>$O/shapes_$lib.err || { tail -20 $O/shapes_$lib.err; exit 1; }
done
python - $O <<'PY'
import json, sys
o = sys.argv[1]
b = {json.loads(l)["case"]: json.loads(l) for l in open(o + "/shapes_base.jsonl")}
for l in open(o + "/shapes_new.jsonl"):
    n = json.loads(l); c = b[n["case"]]
    print(f"{n['case']:34s} buf {c['buf_us']:7.1f} -> {n['buf_us']:7.1f} us ({c['buf_us'] / n['buf_us'] - 1:+.3f})")
PY
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export ARBIUS_KERNEL_LIB=libarbius_kernels_base.so; else unset ARBIUS_KERNEL_LIB; fi
    timeout -k 10 400 python bench.py --steps 6 --warmup 2 > $O/sd_${lib}_$r.log 2>$O/sd_${lib}_$r.err || { tail -20 $O/sd_${lib}_$r.err; exit 1; }
    echo "sd $lib $(tail -1 $O/sd_${lib}_$r.log | cut -c1-110)"
    timeout -k 10 400 python bench.py --model kandinsky2 --steps 4 --warmup 1 > $O/k2_${lib}_$r.log 2>$O/k2_${lib}_$r.err || { tail -20 $O/k2_${lib}_$r.err; exit 1; }
    echo "k2 $lib $(tail -1 $O/k2_${lib}_$r.log | cut -c1-110)"
  done
done
echo "== done $(date +%T)"
