#!/bin/bash
# GEMM + model parity tests, then same-box bench A/B against ab/libmmt_old.so (MMT_LIB_AB)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_nt256_gpu.py tests/test_octo_gpu.py tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ab.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/ab_new$i.log 2>&1 &&
  MMT_LIB_AB=ab/libmmt_old.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/ab_old$i.log 2>&1 || exit 1
done
