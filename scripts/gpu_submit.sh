#!/bin/bash
# usage: gpu_try.sh LOG TIMEOUT CMD  - re-submits only while gpurun reports rc=3 (no box / slot: nothing ran)
LOG=$1; TO=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  echo "rc=$rc try=$i" >> $LOG
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
