#!/bin/bash
# kernel A/B timings + PMC counters for the attention and conv kernels (own run, no tracing domains)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m arbius_amd.ops.build > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python scripts/kernel_ab.py all > gpurun_out/kernel_ab.log 2>&1 || { tail -20 gpurun_out/kernel_ab.log; exit 1; }
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_attn -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/kernel_ab.py attn > $GRAFT_REPO_ROOT/gpurun_out/pmc_attn.log 2>&1
echo done
