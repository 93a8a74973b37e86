#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ntvar
mkdir -p $O
for v in 4 5 6 7; do
  timeout -k 10 300 python tools/gemm_bench.py --variant=$v > $O/gb_$v.log 2>&1 || exit 1
  grep "fwd NT\|dX NN" $O/gb_$v.log | sed "s/^/v$v /"
done
