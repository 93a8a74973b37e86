#!/bin/bash
# the T5 encoder's four products at M = 16,384 under kernel-choice knobs (tools/t5_lib_probe.py)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/t5_gemm_variants.txt
for v in "MMT_X=0" "MMT_NTWS=2" "MMT_NTWS=0" "MMT_GEMM_VARIANT=4" "MMT_GEMM_VARIANT=5" "MMT_GEMM_VARIANT=6"; do
  echo "== $v" >> gpurun_out/t5_gemm_variants.txt
  env $v timeout -k 10 120 python tools/t5_lib_probe.py 2>&1 | grep "M=" >> gpurun_out/t5_gemm_variants.txt || exit 1
done
