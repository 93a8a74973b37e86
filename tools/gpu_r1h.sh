#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/r1h_gb.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_octo_gpu.py tests/test_gemm_gpu.py > gpurun_out/r1h_tests.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r1h_bench.log 2>&1
