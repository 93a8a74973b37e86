#!/bin/bash
# T5 next-step overlap A/B (distributed.DDPStep txt_next): the fork variants in VARIANTS,
# interleaved, at the batches in BATCHES
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/t5_ab.txt
for B in ${BATCHES:-128 512}; do
  for r in 1 2; do
    for v in ${VARIANTS:-MMT_T5_PIPELINE=0 MMT_T5_FORK=bwd MMT_T5_FORK=fwd}; do
      env $v timeout -k 10 300 python bench.py --batch $B --steps 40 --warmup 10 --no-cpu-baseline --no-probes > gpurun_out/t5ab.log 2>&1 || exit 1
      echo "B=$B $v round $r $(grep -o '"value": [0-9.]*' gpurun_out/t5ab.log) $(grep -o '"host_ms_per_step_call": [0-9.]*' gpurun_out/t5ab.log)" >> gpurun_out/t5_ab.txt
    done
  done
done
