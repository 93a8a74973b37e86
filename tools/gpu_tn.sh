#!/bin/bash
# TN weight-gradient kernel: GEMM tests, dW probe A/B (MMT_TN_DMA=0: register-staged kernel), bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/tn_t.log 2>&1 || exit 1
for v in 1 0 1 0; do
  MMT_TN_DMA=$v timeout -k 10 120 python tools/gemm_bench.py --b=512 > gpurun_out/tn_gb$v.log 2>&1 || exit 1
done
for i in 1 2; do
  MMT_TN_DMA=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/tn_new$i.log 2>&1 &&
  MMT_TN_DMA=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/tn_old$i.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_octo_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tn_t2.log 2>&1
