#!/bin/bash
set -o pipefail
export TMPDIR=/tmp MMT_W384_MT=256
mkdir -p gpurun_out
timeout -k 10 120 python tools/w384_probe.py > gpurun_out/wabl_0.log 2>&1 || exit 1
for n in 1 2 3; do
  MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_abl$n.so timeout -k 10 120 python tools/w384_probe.py > gpurun_out/wabl_$n.log 2>&1 || exit 1
done
