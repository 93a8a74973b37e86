#!/bin/bash
# BASELINE configs[3] / configs[4] (OCTO-base 2-cam, OCTO-base hi-res ToMe r=32 fp8) at B = 32:
# bench lines (with the block-0 probes, incl. the fp8 GEMM probe and its bf16 twin), the fp8 path
# A/B (--set fp8=0), and rocprofv3 kernel stats of each step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--batch 32 --no-cpu-baseline"
timeout -k 10 400 python bench.py --config octo-base-2cam $B --steps 30 --warmup 5 > gpurun_out/base2cam.log 2>&1 &&
timeout -k 10 400 python bench.py --config octo-base-hires-tome32 $B --steps 30 --warmup 5 > gpurun_out/hires.log 2>&1 &&
timeout -k 10 400 python bench.py --config octo-base-hires-tome32 $B --steps 30 --warmup 5 --no-probes --set fp8=0 > gpurun_out/hires_bf16.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base2cam -o run --output-format csv -- python bench.py --config octo-base-2cam $B --steps 5 --warmup 2 --no-probes > gpurun_out/prof_base2cam.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hires -o run --output-format csv -- python bench.py --config octo-base-hires-tome32 $B --steps 5 --warmup 2 --no-probes > gpurun_out/prof_hires.log 2>&1
