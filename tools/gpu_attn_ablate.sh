#!/bin/bash
# resident attention forward: per-feature timing of the normal build and of the ablation builds
# (tools/build_abl.sh: 1 = no tile loop, 2 = no K/V DMA, 3 = no O stores)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/attn_ablate.py > gpurun_out/attn_ablate.log 2>&1 &&
for n in 1 2 3; do
  MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_abl$n.so timeout -k 10 300 python tools/attn_ablate.py > gpurun_out/attn_ablate_$n.log 2>&1 || exit 1
done
