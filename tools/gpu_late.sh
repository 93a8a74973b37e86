#!/bin/bash
# late-session batch: register-staged B TN variant A/B ($1) and the B = 128 split A/B
set -eo pipefail
bash tools/gpu_tn_breg.sh $1
cp gpurun_out/ab_MMT_LIB_AB.txt gpurun_out/breg_step_ab.txt
bash tools/gpu_b128_split.sh
