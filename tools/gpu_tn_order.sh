#!/bin/bash
# TN issue order by shape: GEMM tests, dW shapes vs an A/B build ($1) interleaved, step A/B
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_deterministic_gpu.py > gpurun_out/tn_test.log 2>&1
MMT_TN_DEEP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "tn or wgrad or split" > gpurun_out/tn_test_deep.log 2>&1
bash tools/gpu_wgrad_ab2.sh $1
rm -f gpurun_out/ab_MMT_LIB_AB*
bash tools/gpu_ab_env.sh MMT_LIB_AB "multi_modal_transformers_tokenmerge_amd/libmmt_hip.so $1" 2
