#!/bin/bash
# round-4 closing run: whole GPU suite + smoke, the measurement set (PMC passes, bench line,
# rocprof of bench and step), every BASELINE config, the batch sweep
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_all.sh && echo "suite ok" > gpurun_out/final2_rc.txt &&
bash tools/gpu_measure.sh r04h_b512 && echo "measure ok" >> gpurun_out/final2_rc.txt &&
bash tools/gpu_configs.sh && echo "configs ok" >> gpurun_out/final2_rc.txt &&
BATCHES="64 128 256 512" bash tools/gpu_batch_sweep.sh && echo "sweep ok" >> gpurun_out/final2_rc.txt
