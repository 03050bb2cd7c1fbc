#!/bin/bash
# exit-time segfault hunt: the same stream pattern without and with task_stream, markers per step
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5exit}; mkdir -p $O
for m in plain side task; do
  timeout -k 10 120 python -u scripts/exit_probe.py $m > $O/$m.log 2>&1; rc=$?
  echo "mode $m rc=$rc"; cat $O/$m.log | grep -v amdgpu.ids
  [ $rc -ne 0 ] && exit 1
done
exit 0
