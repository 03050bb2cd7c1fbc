#!/bin/bash
# Round-4 A/B call 3: VAE graph replay in the real bench (2 and 4 streams, interleaved), the
# group-of-8 family re-tune with its bench A/B, and the SD1.5 PMC pass + 4-stream kernel summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab3}
mkdir -p $O
export TMPDIR=/tmp
echo "== stag2 tests + A/B $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "stag2 or tile or families" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u scripts/stag2_pd_ab.py --rounds 5 > $O/stag2_ab.jsonl 2>$O/stag2_ab.err || { tail -20 $O/stag2_ab.err; exit 1; }
cut -c1-260 $O/stag2_ab.jsonl
for c in 4 2; do
  for v in 0 1 0 1; do
    echo "== bench c$c vae_graph=$v $(date +%T)"
    ARB_VAE_GRAPH=$v timeout -k 10 400 python bench.py --steps 6 --warmup 2 --concurrent $c > $O/vg_c${c}_$v.log 2>$O/vg_c${c}_$v.err \
      || { tail -20 $O/vg_c${c}_$v.err; exit 1; }
    tail -1 $O/vg_c${c}_$v.log | cut -c1-150
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['stage_s'])" $O/vg_c${c}_$v.log
  done
done
for v in eager graph; do
  a=""; [ $v = graph ] && a="--vae-graph"
  timeout -k 10 400 python -u scripts/graph_serialisation.py $a --groups 3 --json $O/graph_ser_$v.json > $O/graph_ser_$v.log 2>&1 \
    || { tail -20 $O/graph_ser_$v.log; exit 1; }
  head -1 $O/graph_ser_$v.log | cut -c1-400
done
BATCH=16 CONC=2 BENCH_ARGS="--steps 6 --warmup 2 --concurrent 2 --group 8" bash scripts/gpu_retune.sh ${2:-tune16}
