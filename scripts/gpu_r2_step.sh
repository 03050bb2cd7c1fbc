#!/bin/bash
# GN fused-apply A/B + kernel tests, model profiles (RVM, zeroscope, K2), SD bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-step}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/conv_lab.py gnapply > $O/gnapply.log 2>&1 || { tail -20 $O/gnapply.log; exit 1; }
cat $O/gnapply.log | grep gn_apply
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $O/bench_sd.log 2>&1 || { tail -20 $O/bench_sd.log; exit 1; }
tail -1 $O/bench_sd.log | cut -c1-200
MODELS="${MODELS:-robust_video_matting zeroscopev2xl kandinsky2}" bash scripts/gpu_prof_models.sh ${TAG:-step}/prof || exit 1
echo done
