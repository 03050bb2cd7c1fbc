#!/bin/bash
# Op-class ablation inside the deployed 4-stream SD1.5 mix (ARBIUS_EXPERIMENT_SKIP: the class's
# kernels are not launched): what each class really costs when four task streams share the chip.
set -o pipefail
O=gpurun_out/${1:-r5abl}; mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-none shortk geglu gemmbig conv3 attn gnstats,gnapply lnorm vae none}; do
  if [ $v = none ]; then unset ARBIUS_EXPERIMENT_SKIP; else export ARBIUS_EXPERIMENT_SKIP=$v; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "$v $(tail -1 $O/b_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
