#!/bin/bash
# SD1.5 split-K study for the deployed groups of 8 (cold weights; group: batch 16 x 3 copies; solo: batch 2),
# every split.  Input for a re-plan that trades group throughput against solo latency (scripts/split_plan.py).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-sdsplit}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u scripts/split_study.py --model anythingv3 --max-m 100000 --cold --conc 3 --group-size 8 \
  --out $O/sd_split.jsonl > $O/study.log 2>&1 || { tail -5 $O/study.log; exit 1; }
tail -1 $O/study.log | cut -c1-200
