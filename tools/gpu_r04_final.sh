#!/bin/bash
# round-4 final numbers: the bench line (default contract; traffic from the committed PMC file of
# these sources), the attention SQ counter passes, the batch sweep and every BASELINE config
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r04f_bench.log 2>&1; echo "bench $?" > gpurun_out/r04f_rc.txt
bash tools/gpu_attn_pmc.sh; echo "attn_pmc $?" >> gpurun_out/r04f_rc.txt
BATCHES="64 128 256 512" bash tools/gpu_batch_sweep.sh; echo "sweep $?" >> gpurun_out/r04f_rc.txt
bash tools/gpu_configs.sh; echo "configs $?" >> gpurun_out/r04f_rc.txt
