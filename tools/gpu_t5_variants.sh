#!/bin/bash
# the frozen T5 encoder alone at B = 512 under several mmt_gemm kernel choices (MMT_GEMM_VARIANT:
# unset = the dispatch, 8 = gemm_ntw_kernel wherever it applies, 5 / 6 = nt256 with 256 / 192-wide
# tiles), each as a rocprofv3 kernel trace; per-product times: tools/t5_products.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in auto 8 5 6; do
  if [ $v = auto ]; then unset MMT_GEMM_VARIANT; else export MMT_GEMM_VARIANT=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/t5v_$v -o run --output-format csv -- python tools/t5_encoder_probe.py --reps=5 > gpurun_out/t5v_$v.log 2>&1 || exit 1
done
