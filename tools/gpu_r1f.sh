#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r1f_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r1f_bench.log 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r1f_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r1f_prof.log 2>&1
