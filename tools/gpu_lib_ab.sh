#!/bin/bash
# step throughput A/B of libmmt_hip.so against a second build (MMT_LIB_AB=$AB), interleaved rounds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=${AB:-multi_modal_transformers_tokenmerge_amd/libmmt_hip_base.so}
rm -f gpurun_out/lib_ab.txt
for r in 1 2; do
  for v in new base; do
    if [ $v = new ]; then E=""; else E="MMT_LIB_AB=$AB"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-probes --steps 40 --warmup 10 "$@" > gpurun_out/lib_ab_$v$r.log 2>&1 || exit 1
    echo "$v round $r $(grep -o '"value": [0-9.]*' gpurun_out/lib_ab_$v$r.log)" >> gpurun_out/lib_ab.txt
  done
done
