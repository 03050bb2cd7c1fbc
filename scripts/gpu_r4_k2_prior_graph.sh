#!/bin/bash
# Kandinsky2 2 x 4 with / without the diffusion-prior hipGraph (bitwise-equal paths), interleaved.
set -o pipefail
O=gpurun_out/k2pg; mkdir -p $O
for r in 1 2; do
  for g in 1 0; do
    ARB_PRIOR_GRAPH=$g timeout -k 10 400 python bench.py --model kandinsky2 --steps 4 --warmup 1 > $O/g${g}_$r.log 2> $O/g${g}_$r.err || { tail -20 $O/g${g}_$r.err; exit 1; }
    echo "prior_graph=$g run$r $(tail -1 $O/g${g}_$r.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_task_latency_ms"], d["stage_s"])')"
  done
done
