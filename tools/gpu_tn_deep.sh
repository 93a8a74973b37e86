#!/bin/bash
# TN weight-gradient kernel: 2-stage 64-token K-steps (default) vs 4-stage 32-token (MMT_TN_DEEP=1):
# GEMM tests under both, the dW shapes (tools/wgrad_bench.py), step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_deterministic_gpu.py > gpurun_out/tn_test.log 2>&1 &&
MMT_TN_DEEP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_deterministic_gpu.py > gpurun_out/tn_test_deep.log 2>&1 &&
timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/wg_base.log 2>&1 &&
MMT_TN_DEEP=1 timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/wg_deep.log 2>&1 &&
rm -f gpurun_out/ab_MMT_TN_DEEP* &&
bash tools/gpu_ab_env.sh MMT_TN_DEEP "0 1" 2
