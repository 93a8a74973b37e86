#!/bin/bash
# attention GPU tests, then the kernel micro-benchmark with the K/V-resident forward on and off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/attn_debug.py > gpurun_out/attn_debug.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_attn_norm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_test.log 2>&1 &&
timeout -k 10 200 python tools/attn_bench.py --b=512 --L=292,276,212,132,116 > gpurun_out/attn_bench_res.log 2>&1 &&
MMT_ATTN_RES=0 MMT_ATTN_RES_BWD=0 timeout -k 10 200 python tools/attn_bench.py --b=512 --L=292,276,212,132,116 > gpurun_out/attn_bench_old.log 2>&1
