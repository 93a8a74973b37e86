#!/bin/bash
# MLP up on the activation-stationary kernel with the relu-bit image: parity tests, kernel bench,
# step A/B (MMT_XS=1: bias-only products only, as round 4; 2: also the MLP up)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemm_nt256_gpu.py -k "activation_stationary or relu_bits or keep_bits or ntws" > gpurun_out/xs_rb_test.log 2>&1 &&
timeout -k 10 200 python tools/xs_bench.py > gpurun_out/xs_rb_bench.log 2>&1 &&
rm -f gpurun_out/ab_MMT_XS* &&
bash tools/gpu_ab_env.sh MMT_XS "1 2" 2
