#!/bin/bash
# round 2: RVM forks (tests + bench at two task slots), then PMC passes on the level-0 conv tiles
set -o pipefail
TAG=r2rvm2 bash $GRAFT_REPO_ROOT/scripts/gpu_r2_rvm2.sh && TAG=r2pmc bash $GRAFT_REPO_ROOT/scripts/gpu_r2_pmc.sh
