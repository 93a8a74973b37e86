#!/bin/bash
# fp8 activation-stationary kernel: tests, then configs[4] with fp8 on / off
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--batch 32 --no-cpu-baseline"
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp8_test.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_octo_gpu.py -k "hires or base_2cam" -x -q --timeout 250 --timeout-method thread > gpurun_out/fp8_parity.log 2>&1 &&
timeout -k 10 400 python bench.py --config octo-base-hires-tome32 $B --steps 30 --warmup 5 > gpurun_out/hires.log 2>&1 &&
timeout -k 10 400 python bench.py --config octo-base-hires-tome32 $B --steps 30 --warmup 5 --no-probes --set fp8=0 > gpurun_out/hires_bf16.log 2>&1
