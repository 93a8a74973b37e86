#!/bin/bash
# nt256 GEMM: numerics, then old (variant 4, 128x128 glds) vs new (auto / forced BN) timings.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_nt256_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_tests.log 2>&1 &&

timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/nt_gbauto.log 2>&1 &&
timeout -k 10 200 python tools/gemm_bench.py --variant=6 > gpurun_out/nt_gb6.log 2>&1
