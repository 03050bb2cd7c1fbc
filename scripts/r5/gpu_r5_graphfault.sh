#!/bin/bash
# the SIGSEGV inside CUDAGraph::replay under rocprofv3 and the VAE-graph stall.
# 1. traced bench with HIP graph packet capture OFF (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0): does the fault go?
# 2. untraced VAE-graph bench, packet capture on / off, vs the eager-VAE default: is the stall the same path?
# 3. traced default bench with /proc/self/maps dumped after warm-up (the run that faulted before): the
#    crash stack's return addresses are symbolised offline against the same image's libraries.
# A native fault ends the script (last step on purpose).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r5gf}; mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
echo "load $(cat /proc/loadavg)"
val() { tail -1 $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_s"])'; }
(cd /tmp && DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p0 -o run -- python3 $R/bench.py --steps 4 --warmup 1 > $O/trace_nocap.log 2> $O/trace_nocap.err) || { tail -30 $O/trace_nocap.err; exit 1; }
echo "traced nocapture: $(val $O/trace_nocap.log)"
rm -rf $O/p0
for v in vae_cap vae_nocap eager_nocap default; do
  unset ARB_VAE_GRAPH DEBUG_CLR_GRAPH_PACKET_CAPTURE
  case $v in vae_cap) export ARB_VAE_GRAPH=1;; vae_nocap) export ARB_VAE_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0;;
    eager_nocap) export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0;; esac
  timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 > $O/b_$v.log 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  echo "$v $(val $O/b_$v.log)"
done
unset ARB_VAE_GRAPH DEBUG_CLR_GRAPH_PACKET_CAPTURE
(cd /tmp && ARB_DUMP_MAPS=$O/maps.txt timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p1 -o run -- python3 $R/bench.py --steps 4 --warmup 1 > $O/trace_cap.log 2> $O/trace_cap.err) || { tail -40 $O/trace_cap.err; rm -rf $O/p1; exit 1; }
echo "traced default: $(val $O/trace_cap.log)"
rm -rf $O/p1
