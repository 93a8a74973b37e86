#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_nt256_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1 &&
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/nt_gbauto.log 2>&1 &&
timeout -k 5 60 ./tools/nt_trace 70656 1536 384 5 > gpurun_out/nttrace1.log 2>&1 &&
timeout -k 5 60 ./tools/nt_trace 4096 4096 4096 5 >> gpurun_out/nttrace1.log 2>&1
