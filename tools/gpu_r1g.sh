#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_attn_norm_gpu.py tests/test_octo_gpu.py tests/test_t5_stem_gpu.py > gpurun_out/r1g_tests.log 2>&1 &&
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/r1g_attn.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r1g_bench.log 2>&1
