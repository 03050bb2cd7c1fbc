#!/bin/bash
# After the re-pin: every GPU test against the committed pins, the smoke, and the default bench; then
# the stag2 prefetch A/B, VAE-graph serialisation probe, K2 prior-graph A/B and zeroscope evidence.
set -o pipefail
R=$GRAFT_REPO_ROOT
SKIP_PROF=1 bash scripts/gpu_check.sh ${1:-chk4} && bash scripts/gpu_r4_video_graph.sh ${2:-vidg}
