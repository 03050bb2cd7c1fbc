#!/bin/bash
# Cold-weight family study at the pinned splits (bitwise-neutral candidates): SD1.5 group side (batch 8,
# 4 concurrent copies) and Kandinsky2 solo + group sides (scripts/split_study.py --cold --keep-split).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-coldfam}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 560 python3 -u scripts/split_study.py --model anythingv3 --max-m 100000 --only group --keep-split \
  --cold --out $O/sd_group.jsonl > $O/sd.log 2>&1 || { tail -5 $O/sd.log; exit 1; }
tail -1 $O/sd.log | cut -c1-200
timeout -k 10 560 python3 -u scripts/split_study.py --model kandinsky2 --max-m 100000 --keep-split --cold \
  --out $O/k2_both.jsonl > $O/k2.log 2>&1 || { tail -5 $O/k2.log; exit 1; }
tail -1 $O/k2.log | cut -c1-200
