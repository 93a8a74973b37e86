#!/bin/bash
# Round-end measurements: bench line (with the CPU baseline) and rocprofv3 kernel-trace summaries
# of the bench and of the probe GEMM.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_probe -o run --output-format csv -- python bench.py --probe-only > $O/prof_probe.log 2>&1
