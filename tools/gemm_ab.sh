#!/bin/bash
# GEMM unit tests under each main-loop variant, then the micro-benchmark per variant
# (mmt_gemm_set_variant: 0 = double-buffered one-tile workgroups, 1 = persistent single stage,
# 3 = chosen by K-steps).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 3 0 1; do
  MMT_GEMM_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/gemm_t$v.log 2>&1 || exit 1
done
for v in 3 0 1; do
  timeout -k 10 200 python tools/gemm_bench.py --variant=$v > gpurun_out/gb$v.log 2>&1 || exit 1
done
for v in 0 1; do
  timeout -k 10 200 python tools/gemm_bench.py --sweep --variant=$v > gpurun_out/sw$v.log 2>&1 || exit 1
done
