#!/bin/bash
# Stream-serialisation evidence: rocprofv3 kernel traces of the 2-stream SD1.5 bench with the VAE
# eager (default) and replayed as a hipGraph (ARB_VAE_GRAPH=1), summarised per stream
# (scripts/stream_timeline.py): busy time, idle gaps, and what the other stream runs meanwhile.
set -o pipefail
TAG=${1:-gtrace}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-default vaegraph}; do
  echo "== trace $v $(date +%T)"
  if [ $v = vaegraph ]; then export ARB_VAE_GRAPH=1; else unset ARB_VAE_GRAPH; fi
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 \
     --concurrent ${CONC:-2} > $O/trace_$v.log 2>&1) || { tail -20 $O/trace_$v.log; exit 1; }
  grep metric $O/trace_$v.log | cut -c1-140
  python scripts/stream_timeline.py $O/p_$v/run_results.db --md $O/timeline_$v.md | head -12
  rm -rf $O/p_$v
done
echo "== done $(date +%T)"
