#!/bin/bash
# Interleaved min-of-N A/B of encoder builds (scripts/h264_bench.cpp): prints min ms/frame per binary
# and checks that every binary wrote the same bytes (FNV of all NALs).
#   scripts/h264_ab.sh N FRAMES bin1 bin2 ...
N=$1; FR=$2; shift 2
declare -A best fnv
for i in $(seq $N); do
  for b in "$@"; do
    line=$($b $FR) || exit 1
    ms=$(echo "$line" | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_frame"])')
    f=$(echo "$line" | python3 -c 'import json,sys; print(json.load(sys.stdin)["fnv"])')
    fnv[$b]=$f
    if [ -z "${best[$b]}" ] || python3 -c "import sys; sys.exit(0 if $ms < ${best[$b]} else 1)"; then best[$b]=$ms; fi
  done
done
for b in "$@"; do echo "$b min_ms_per_frame=${best[$b]} fnv=${fnv[$b]}"; done
