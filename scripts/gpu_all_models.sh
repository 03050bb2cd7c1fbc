#!/bin/bash
# One bench line per BASELINE config (SD default, SD latency mode, Kandinsky2, zeroscope, RVM).
set -o pipefail
TAG=${1:-allm}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 500 python bench.py "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -20 $O/$name.log; exit 1; }
  tail -1 $O/$name.log > $O/$name.json
  echo "$name $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["unit"], d.get("p50_task_latency_ms"))' $O/$name.json)"
}
run sd15_default
run sd15_latency --concurrent 1 --group 1
run k2_default --model kandinsky2 --steps 2 --warmup 1
run zeroscope --model zeroscopev2xl --steps 2 --warmup 1
run rvm --model robust_video_matting --steps 3 --warmup 1
