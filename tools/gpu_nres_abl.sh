#!/bin/bash
# residual-stream kernel ablations (tools/build_abl_nres.sh) on the Dense_1 / out-projection probes
set -o pipefail
export TMPDIR=/tmp MMT_NRES=2
mkdir -p gpurun_out
echo "== base" >> gpurun_out/nres_abl.txt
timeout -k 10 120 python tools/res_probe.py >> gpurun_out/nres_abl.txt 2>&1 || exit 1
for n in "$@"; do
  echo "== abl $n" >> gpurun_out/nres_abl.txt
  MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_nresabl$n.so timeout -k 10 120 python tools/res_probe.py >> gpurun_out/nres_abl.txt 2>&1 || exit 1
done
