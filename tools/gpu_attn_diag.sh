#!/bin/bash
# resident attention diagnosis: feature timing (plain / mask / dropout), ablation builds given as
# arguments (tools/build_abl.sh), then the SQ / HBM counter passes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/attn_ablate.py > gpurun_out/attn_features.log 2>&1 &&
bash tools/gpu_attn_ablate.sh "$@" &&
bash tools/gpu_attn_pmc.sh
