#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_attn_norm_gpu.py tests/test_octo_gpu.py -q -x > gpurun_out/attn_t.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r1_bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
