#!/bin/bash
# GEMM unit tests under each main-loop variant, micro-benchmark per variant, phase traces.
# (mmt_gemm_set_variant: 0 = PIPE 0 / BK 64, 1 = PIPE 1 / BK 64, 2 = PIPE 1 / BK 128, -1 auto)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2; do
  MMT_GEMM_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gemm_gpu.py -q -x > gpurun_out/gemm_t$v.log 2>&1 || exit 1
done
for v in 0 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --variant=$v > gpurun_out/gb$v.log 2>&1 || exit 1
done
for v in 1 2; do
  for s in "18688 384 384" "18688 1536 384" "18688 384 1536"; do
    timeout -k 5 60 ./tools/gemm_trace $s $v || exit 1
  done
done > gpurun_out/trace.log 2>&1
