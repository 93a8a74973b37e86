#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace -d gpurun_out/l2a -o run --output-format csv -- python tools/gemm_bench.py --variant=1 > gpurun_out/l2a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/l2b -o run --output-format csv -- python tools/gemm_bench.py --variant=1 > gpurun_out/l2b.log 2>&1
