#!/bin/bash
# Zeroscope: re-tune the video plan table's tile families at the planned split-K (bitwise: every candidate
# is checked against the planned kernel's output) over the current families incl. stag2 192x192 (cfg 45),
# two concurrent copies; then a same-box A/B of the tuned table (ARB_CONV_PLANS) against the built-in one.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5zs}; mkdir -p $O
export TMPDIR=/tmp
echo "load $(cat /proc/loadavg)"
timeout -k 10 700 python -u scripts/tune_family.py $O/plans.inc --plans --models video --conc 2 \
  --families ${FAMS:-20,21,22,23,32,33,34,35,36,37,38,39,40,41,42,43,44,45} > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
grep -c "^plan" $O/tune.log; grep "^plan" $O/tune.log | awk '{print $0}' | head -60 | cut -c1-120
for v in base tuned base tuned; do
  if [ $v = tuned ]; then export ARB_CONV_PLANS=$O/plans.inc; else unset ARB_CONV_PLANS; fi
  timeout -k 10 300 python3 bench.py --model zeroscopev2xl --steps 3 --warmup 1 > $O/zs_$v.log 2> $O/zs_$v.err || { tail -20 $O/zs_$v.err; exit 1; }
  echo "zs $v $(tail -1 $O/zs_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
