#!/bin/bash
# resident attention: kernel timing of the normal build and of the ablation builds given as
# arguments (tools/build_abl.sh: fwd 1 = no tile loop, 2 = no K/V DMA, 3 = no O stores;
# bwd 4 = no phase-A tiles, 5 = no phase-B tiles, 6 = no DMA)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/attn_bench.py --b=512 --L=292,212,116 > gpurun_out/attn_abl_base.log 2>&1 || exit 1
for n in "$@"; do
  MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_abl$n.so timeout -k 10 200 python tools/attn_bench.py --b=512 --L=292,212,116 > gpurun_out/attn_abl_$n.log 2>&1 || exit 1
done
