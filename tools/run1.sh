#!/bin/bash
# GPU-box check: parity tests, then a short bench, then a kernel-trace profile.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r1_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/r1_bench.log 2>&1 &&
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gb.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
rc=$?
echo "exit $rc" >> gpurun_out/r1_tests.log
exit $rc
