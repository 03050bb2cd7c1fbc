#!/bin/bash
# SD1.5 family re-tune at batch 8 under 4 concurrent copies (the deployed 4 x 4), restricted to the
# K-half staggered tiles incl. stag2 192x192 (cfg 45, added after the round-4 tune) + each shape's kept
# family; merged onto the built-in table; then a same-box SD bench A/B (ARB_CONV_FAMILY).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5sdt}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
timeout -k 10 ${TUNE_S:-600} python -u scripts/tune_family.py $O/f.inc --batch 8 --conc 4 --models sd15 \
  --families ${FAMS:-42,43,44,45} --merge arbius_amd/ops/csrc/conv_family.inc > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep -E "re-tuned" $O/tune.log | head -30
for v in base tuned base tuned; do
  if [ $v = tuned ]; then export ARB_CONV_FAMILY=$O/f.inc; else unset ARB_CONV_FAMILY; fi
  timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 > $O/sd_$v.log 2> $O/sd_$v.err || { tail -20 $O/sd_$v.err; exit 1; }
  echo "sd $v $(tail -1 $O/sd_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
