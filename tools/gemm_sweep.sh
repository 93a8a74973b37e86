#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_bench.py --sweep --variant=0 > gpurun_out/sw0.log 2>&1 &&
timeout -k 10 200 python tools/gemm_bench.py --sweep --variant=1 > gpurun_out/sw1.log 2>&1 &&
timeout -k 10 200 python tools/gemm_bench.py --sweep --variant=2 > gpurun_out/sw2.log 2>&1
