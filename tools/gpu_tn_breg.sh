#!/bin/bash
# TN kernel with register-staged B pieces (A/B build $1): GEMM tests on it, dW shapes and step
# interleaved against the default build
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
MMT_LIB_AB=$1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/breg_test.log 2>&1
bash tools/gpu_wgrad_ab2.sh $1
rm -f gpurun_out/ab_MMT_LIB_AB*
bash tools/gpu_ab_env.sh MMT_LIB_AB "multi_modal_transformers_tokenmerge_amd/libmmt_hip.so $1" 2
