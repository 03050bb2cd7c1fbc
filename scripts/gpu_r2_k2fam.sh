#!/bin/bash
# round 2: tile families for the Kandinsky2 (mainnet model) lock-step batch-8 shapes under two
# concurrent task streams, plus the K2 bench line they will be compared against
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2k2f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/tune_family.py $O/conv_family.inc --models kandinsky2 --batch 8 --conc 2 --merge arbius_amd/ops/csrc/conv_family.inc > $O/tune_family_k2.log 2>&1 || { tail -30 $O/tune_family_k2.log; exit 1; }
grep -c "canonical" $O/tune_family_k2.log
timeout -k 10 600 python bench.py --model kandinsky2 --steps 3 --warmup 1 > $O/bench_k2.json 2> $O/bench_k2.err || { tail -20 $O/bench_k2.err; exit 1; }
cat $O/bench_k2.json
