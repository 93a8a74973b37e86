#!/bin/bash
# Residual-stream GEMM probes (tools/res_probe.py) under each kernel choice:
#   MMT_NRES 0 = 128 x 128 kernel / narrow kernel, 1 = gemm_nres_kernel for the fp32 products,
#   2 = also the plain bf16 product; MMT_NRES_W = weight path (0 LDS-DMA, 1 VGPR + ds_write)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "MMT_NRES=0" "MMT_NRES=2 MMT_NRES_W=0"; do
  echo "== $cfg" >> gpurun_out/res_probe.txt
  env $cfg timeout -k 10 120 python tools/res_probe.py >> gpurun_out/res_probe.txt 2>&1 || exit 1
done
