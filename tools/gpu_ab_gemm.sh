#!/bin/bash
# GEMM tests, gemm_bench A/B (in-tree vs ab/libmmt_old.so), bench A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_nt256_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/abg_t.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python tools/gemm_bench.py --b=512 > gpurun_out/abg_gb_new$i.log 2>&1 &&
  MMT_LIB_AB=ab/libmmt_old.so timeout -k 10 120 python tools/gemm_bench.py --b=512 > gpurun_out/abg_gb_old$i.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/abg_new$i.log 2>&1 &&
  MMT_LIB_AB=ab/libmmt_old.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/abg_old$i.log 2>&1 || exit 1
done
