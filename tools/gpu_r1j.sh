#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_attn_norm_gpu.py tests/test_octo_gpu.py > gpurun_out/r1j_tests.log 2>&1 &&
timeout -k 10 200 python tools/attn_bench.py > gpurun_out/r1j_attn.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r1j_bench.log 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r1j_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r1j_prof.log 2>&1
