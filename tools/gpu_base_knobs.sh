#!/bin/bash
# GEMM routing knobs at BASELINE configs[3] (octo-base-2cam, B = 32): MMT_NTWS 1 (default) / 0 / 2
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_MMT_NTWS*
bash tools/gpu_ab_env.sh MMT_NTWS "1 0 2" 2 --config octo-base-2cam --batch 32 --steps 30 --warmup 5
