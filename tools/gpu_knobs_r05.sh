#!/bin/bash
# round-5 knob A/Bs, one box: hipBLASLt for the plain products at B = 512, the dW side-stream
# per-block join (lag) at B = 128
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_MMT_BLASLT.txt gpurun_out/ab_MMT_WGRAD_LAG.txt
bash tools/gpu_ab_env.sh MMT_BLASLT "0 1" 2 --steps 40 --warmup 10 &&
bash tools/gpu_ab_env.sh MMT_WGRAD_LAG "0 1 2" 1 --batch 128 --steps 40 --warmup 10
