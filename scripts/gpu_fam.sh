#!/bin/bash
# Tile-family re-tune at the canonical split (bitwise-neutral: no golden moves) for the lock-step
# batch-8 shapes under 2-stream concurrency, with every family incl. the staggered two-group tiles;
# rebuild with the new table and bench SD1.5 + Kandinsky2.  Also an in-process A/B of the planned
# convs against the previous library build (libarbius_kernels_base.so).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-fam}
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step ab
timeout -k 10 300 python -u scripts/conv_lab.py ab > $O/ab.jsonl 2>$O/ab.err || { tail -20 $O/ab.err; exit 1; }
cut -c1-300 $O/ab.jsonl
step fam_sd
timeout -k 10 900 python -u scripts/tune_family.py $O/fam_sd.inc --batch 8 --conc 2 --models sd15 \
  --merge arbius_amd/ops/csrc/conv_family.inc > $O/fam_sd.log 2>&1 || { tail -20 $O/fam_sd.log; exit 1; }
grep -c canonical $O/fam_sd.log
step fam_k2
timeout -k 10 900 python -u scripts/tune_family.py $O/fam.inc --batch 8 --conc 2 --models kandinsky2 --res 768 \
  --merge $O/fam_sd.inc > $O/fam_k2.log 2>&1 || { tail -20 $O/fam_k2.log; exit 1; }
grep -c canonical $O/fam_k2.log
step build
cp $O/fam.inc arbius_amd/ops/csrc/conv_family.inc && timeout -k 10 600 python -m arbius_amd.ops.build > $O/build.log 2>&1 || { tail $O/build.log; exit 1; }
step bench_sd
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > $O/sd.log 2>$O/sd.err || { tail -20 $O/sd.err; exit 1; }
tail -1 $O/sd.log | cut -c1-200
step bench_k2
timeout -k 10 500 python bench.py --model kandinsky2 > $O/k2.log 2>$O/k2.err || { tail -20 $O/k2.err; exit 1; }
tail -1 $O/k2.log | cut -c1-200
step done
