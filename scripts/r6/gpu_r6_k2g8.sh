#!/bin/bash
# Kandinsky2 lock-step groups of 8: cold-weight family study of the batch-16 launches
# at the pinned splits (4 concurrent copies, bitwise-neutral candidates), the family override it implies,
# then 4 x 4 (default) vs 4 x 8 / 3 x 8 with it, bracketed by the default.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-k2g8}; mkdir -p $O
export TMPDIR=/tmp
echo "== study $(date +%T)"
timeout -k 10 1000 python3 -u scripts/split_study.py --model kandinsky2 --max-m 100000 --only group --keep-split \
  --cold --conc 4 --group-size 8 --out $O/k2_g8.jsonl > $O/study.log 2>&1 || { tail -5 $O/study.log; exit 1; }
python3 scripts/split_plan.py $O/k2_g8.jsonl --out $O/g8 --keep-splits --solo-step-us 1e12 --group-step-us 1000 | tail -2
one() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 500 python3 bench.py --model kandinsky2 "$@" > $O/$n.log 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_task_latency_ms"])')"
}
fam() { ( export ARB_CONV_FAMILY=$O/g8_family.txt; one "$@" ); }
echo "== benches $(date +%T)"
one c4g4 --steps 3 --warmup 1 || exit 1
fam c4g8_fam --concurrent 4 --group 8 --steps 2 --warmup 1 || exit 1
fam c3g8_fam --concurrent 3 --group 8 --steps 2 --warmup 1 || exit 1
one c4g4b --steps 3 --warmup 1 || exit 1
fam c4g8_famb --concurrent 4 --group 8 --steps 2 --warmup 1 || exit 1
echo "== done $(date +%T)"
echo "== aten sites $(date +%T)"
timeout -k 10 400 python3 scripts/aten_gpu_sites.py kandinsky2 --steps 10 > $O/aten_k2.jsonl 2> $O/aten_k2.err || { tail -5 $O/aten_k2.err; exit 1; }
timeout -k 10 400 python3 scripts/aten_gpu_sites.py anythingv3 --steps 10 > $O/aten_sd.jsonl 2> $O/aten_sd.err || { tail -5 $O/aten_sd.err; exit 1; }
grep -h copy_api $O/aten_k2.jsonl $O/aten_sd.jsonl | head -20
echo "== done2 $(date +%T)"
