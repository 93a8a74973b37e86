#!/bin/bash
# GEMM unit tests under each kernel variant, then the micro-benchmark per variant
# (mmt_gemm_set_variant: 0 PIPE 0/BK 64, 1 PIPE 1/BK 64, 2 PIPE 1/BK 128, 3 256x192, 4 glds NT, -1 auto).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 4; do
  MMT_GEMM_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/gemm_t$v.log 2>&1 || exit 1
done
for v in 1 4; do
  timeout -k 10 200 python tools/gemm_bench.py --variant=$v > gpurun_out/gb$v.log 2>&1 || exit 1
done
