#!/bin/bash
# weight-gradient split target at the small per-GPU batch (B = 128)
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_MMT_WGRAD_WGS*
bash tools/gpu_ab_env.sh MMT_WGRAD_WGS "128 64 96 192" 2 --batch 128
