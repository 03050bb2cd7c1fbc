#!/bin/bash
# Zeroscope where-does-the-time-go: deployed 1-stream kernel summary (rocprofv3, graph replay) and the
# ATen call sites left on its eager path (torch.profiler with Python stacks).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-zsprof}; mkdir -p $O
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --model zeroscopev2xl \
  --concurrent 1 --steps 1 --warmup 1 > $O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python scripts/prof_summary.py $O/prof/run_results.db --top 45 --md $O/rocprof_zs.md > /dev/null 2>&1; rm -rf $O/prof
head -25 $O/rocprof_zs.md
timeout -k 10 400 python3 scripts/aten_gpu_sites.py zeroscopev2xl --steps 4 > $O/aten_sites.jsonl 2> $O/aten.err || { tail -20 $O/aten.err; exit 1; }
head -12 $O/aten_sites.jsonl | cut -c1-250
