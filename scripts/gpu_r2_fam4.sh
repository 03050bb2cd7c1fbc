#!/bin/bash
# round 2: tile families for partial lock-step groups (batch 4 = groups of 2 under the batch-8 plans)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2f4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/tune_family.py $O/conv_family.inc --models sd15,kandinsky2 --batch 4 --merge arbius_amd/ops/csrc/conv_family.inc > $O/tune_family4.log 2>&1 || { tail -30 $O/tune_family4.log; exit 1; }
grep -c "canonical" $O/tune_family4.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --concurrent 1 --group 2 > $O/bench_sd_c1g2.json 2> $O/bench_sd_c1g2.err || { tail -20 $O/bench_sd_c1g2.err; exit 1; }
cat $O/bench_sd_c1g2.json
