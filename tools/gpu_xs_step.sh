#!/bin/bash
# step A/B of the activation-stationary QKV GEMM (MMT_XS) at B = 512
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 40 --warmup 10 --no-probes --no-cpu-baseline > gpurun_out/xs_step_on.log 2>&1 &&
MMT_XS=0 timeout -k 10 400 python bench.py --steps 40 --warmup 10 --no-probes --no-cpu-baseline > gpurun_out/xs_step_off.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 40 --warmup 10 --no-probes --no-cpu-baseline > gpurun_out/xs_step_on2.log 2>&1
