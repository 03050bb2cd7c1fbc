#!/bin/bash
# round 2: SD1.5 streams x lock-step group trade-off on the current tree (free-running slots)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2sw}
mkdir -p $O
export TMPDIR=/tmp
for cg in "2 6" "2 8" "3 4" "1 8"; do
  set -- $cg
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --concurrent $1 --group $2 > $O/bench_c$1_g$2.json 2> $O/bench_c$1_g$2.err || { tail -20 $O/bench_c$1_g$2.err; exit 1; }
  cut -c1-160 $O/bench_c$1_g$2.json
done
