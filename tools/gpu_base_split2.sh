#!/bin/bash
# weight-gradient split target (MMT_WGRAD_WGS) at the OCTO-base configs (BASELINE configs[3] / [4])
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_MMT_WGRAD_WGS* gpurun_out/base_split.txt
bash tools/gpu_ab_env.sh MMT_WGRAD_WGS "96 64 128" 2 --config octo-base-2cam --batch 32 --steps 30 --warmup 5
sed 's/^/octo-base-2cam /' gpurun_out/ab_MMT_WGRAD_WGS.txt >> gpurun_out/base_split.txt && rm -f gpurun_out/ab_MMT_WGRAD_WGS.txt
bash tools/gpu_ab_env.sh MMT_WGRAD_WGS "96 128" 1 --config octo-base-hires-tome32 --batch 32 --steps 30 --warmup 5
sed 's/^/octo-base-hires-tome32 /' gpurun_out/ab_MMT_WGRAD_WGS.txt >> gpurun_out/base_split.txt
rm -f gpurun_out/ab_MMT_WGRAD_WGS.txt
