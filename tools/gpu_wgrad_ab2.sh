#!/bin/bash
# dW shapes (tools/wgrad_bench.py) of the default build and an A/B build ($1), interleaved x2
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/wg2_base_$r.log 2>&1
  MMT_LIB_AB=$1 timeout -k 10 200 python tools/wgrad_bench.py > gpurun_out/wg2_ab_$r.log 2>&1
done
