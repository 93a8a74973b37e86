#!/bin/bash
# LayerNorm / ToMe HBM kernels: tests, then the micro-benchmark with the new forms on / off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attn_norm_gpu.py tests/test_tome_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ln_test.log 2>&1 &&
timeout -k 10 120 python tools/ln_bench.py > gpurun_out/ln_new.log 2>&1 &&
MMT_SNB512=0 timeout -k 10 120 python tools/ln_bench.py > gpurun_out/ln_old.log 2>&1
