#!/bin/bash
# round 2: tile-family table for solo (batch 2) shapes at the canonical split, plus the latency bench
# before it is applied (baseline for the A/B after the rebuild)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2fam}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/tune_family.py $O/conv_family.inc > $O/tune_family.log 2>&1 || { tail -30 $O/tune_family.log; exit 1; }
grep -c "canonical" $O/tune_family.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 1 > $O/bench_sd_latency.json 2> $O/bench_sd_latency.err || { tail -20 $O/bench_sd_latency.err; exit 1; }
cat $O/bench_sd_latency.json
