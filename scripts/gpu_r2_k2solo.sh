#!/bin/bash
# round 2: Kandinsky2 solo latency before the K2 solo tile-family table, and the table itself
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2k2s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --model kandinsky2 --steps 3 --warmup 1 --concurrent 1 --group 1 > $O/bench_k2_latency.json 2> $O/bench_k2_latency.err || { tail -20 $O/bench_k2_latency.err; exit 1; }
cat $O/bench_k2_latency.json
timeout -k 10 900 python -u scripts/tune_family.py $O/conv_family.inc --models kandinsky2 --batch 2 --merge arbius_amd/ops/csrc/conv_family.inc > $O/tune_family_k2.log 2>&1 || { tail -30 $O/tune_family_k2.log; exit 1; }
grep -c "canonical" $O/tune_family_k2.log
