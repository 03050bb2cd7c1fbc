#!/bin/bash
# A/B call 5: the VAE hipGraph after removing the memcpy node from the d=512 attention (2 and 4
# streams, interleaved), then the round-4 SD1.5 kernel evidence (PMC pass, 4-stream rocprof summary
# and per-stream timeline).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab5}
mkdir -p $O
export TMPDIR=/tmp
echo "== tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "large_head or vae or attention" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in 4 2; do
  for v in 0 1 0 1; do
    echo "== bench c$c vae_graph=$v $(date +%T)"
    ARB_VAE_GRAPH=$v timeout -k 10 400 python bench.py --steps 6 --warmup 2 --concurrent $c > $O/vg_c${c}_$v.log 2>$O/vg_c${c}_$v.err \
      || { tail -20 $O/vg_c${c}_$v.err; exit 1; }
    tail -1 $O/vg_c${c}_$v.log | cut -c1-150
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['stage_s'])" $O/vg_c${c}_$v.log
  done
done
bash scripts/gpu_r4_profiles.sh ${2:-prof4}
