#!/bin/bash
# Step-throughput A/B of one environment knob, interleaved runs on one box:
#   tools/gpu_ab_env.sh VAR "valA valB" [rounds] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=$1; VALS=$2; ROUNDS=${3:-2}; shift 3
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    tag=$(basename "$v")
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-probes "$@" > gpurun_out/ab_${VAR}_${tag}_$r.log 2>&1 || exit 1
    echo "$VAR=$tag round $r $(grep -o '"value": [0-9.]*' gpurun_out/ab_${VAR}_${tag}_$r.log)" >> gpurun_out/ab_${VAR}.txt
  done
done
