#!/bin/bash
# bench line + kernel-trace profile of the default bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/p_bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/p_prof.log 2>&1
