#!/bin/bash
# Re-tune the pinned conv plans of one model family on the GPU (scripts/autotune_conv.py) under the
# deployed 2-stream concurrency; writes gpurun_out/<tag>/{conv_plans.inc,autotune_conv.json}.
#   MODELS=video bash scripts/gpu_tune.sh zs_tune [extra autotune args]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-tune}
shift
mkdir -p $O
timeout -k 10 1000 python -u scripts/autotune_conv.py $O --models ${MODELS:-video} --conc 2 \
  --merge arbius_amd/ops/csrc/conv_plans.inc "$@" > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
grep -c '"kind"' $O/tune.log
python - "$O/autotune_conv.json" <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
gain = [(x["auto_us"] - x["best_us"], x) for x in r if x["kind"] == "conv" and "auto_us" in x]
print("total auto us %.0f -> best us %.0f" % (sum(x["auto_us"] for _, x in gain), sum(x["best_us"] for _, x in gain)))
for g, x in sorted(gain, key=lambda t: -t[0])[:12]:
    print(x["shape"], x["auto_cfg"], "->", x["best_cfg"], x["best_split"], x["auto_us"], "->", x["best_us"], x["best_tflops"])
PY
