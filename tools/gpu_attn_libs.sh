#!/bin/bash
# attention micro-bench over several builds of the library (interleaved rounds):
#   tools/gpu_attn_libs.sh TAG lib1 lib2 ...   ("default" = libmmt_hip.so, else libmmt_hip_<name>.so)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
out=gpurun_out/${TAG}.txt
rm -f $out
for r in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then E=""; else E="MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_$v.so"; fi
    env $E timeout -k 10 200 python -u tools/attn_bench.py --b=512 --L=292,228,164 > gpurun_out/${TAG}_$v$r.log 2>&1 || exit 1
    grep octo gpurun_out/${TAG}_$v$r.log | sed "s/^/$v r$r /" >> $out
  done
done
