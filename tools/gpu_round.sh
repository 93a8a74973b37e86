#!/bin/bash
# bench line, epilogue ablation and a kernel-trace profile of the step (one gpurun call)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r_bench.log 2>&1 &&
timeout -k 10 200 python tools/epi_bench.py > gpurun_out/r_epi.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r_prof -o run --output-format csv -- python bench.py --steps 9 --warmup 3 --no-cpu-baseline --no-probes > gpurun_out/r_prof.log 2>&1
