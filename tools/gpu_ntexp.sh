#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ntexp
mkdir -p $O
L=multi_modal_transformers_tokenmerge_amd/libmmt_hip.so
for v in def nt def nt; do
  cp tools/_exp/lib_$v.so $L &&
  timeout -k 10 300 python tools/gemm_bench.py > $O/gb_$v.log 2>&1 &&
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit 1
  grep "fwd NT" $O/gb_$v.log | head -3 | sed "s/^/$v /"
  tail -1 $O/bench_$v.log | cut -c80-125 | sed "s/^/$v /"
done
cp tools/_exp/lib_def.so $L
