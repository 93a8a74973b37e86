#!/bin/bash
# per-GPU batch sweep of the bench step (throughput vs B)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/bsweep.log
for b in ${BATCHES:-256 384 512 192 320 256}; do
  timeout -k 10 250 python bench.py --batch $b --steps 40 --warmup 10 --no-cpu-baseline --no-probes > gpurun_out/bs_$b.log 2>&1 || exit 1
  echo "B=$b $(grep -o '"value": [0-9.]*' gpurun_out/bs_$b.log)" >> gpurun_out/bsweep.log
done
