#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gemm_nt256_gpu.py tests/test_gemm_gpu.py tests/test_octo_gpu.py > gpurun_out/r1i_tests.log 2>&1 &&
bash tools/gpu_measure.sh
