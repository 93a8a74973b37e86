#!/bin/bash
# step throughput at several per-GPU batches, interleaved with the metric batch (one box)
set -o pipefail
TAG=${1:-bsweep}
mkdir -p gpurun_out
for b in 512 64 128 256 512; do
  timeout -k 10 300 python -u bench.py --batch $b --steps 40 --warmup 10 --no-cpu-baseline --no-probes > gpurun_out/${TAG}_b$b.log 2>&1 || exit 1
  grep '^{' gpurun_out/${TAG}_b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['ms_per_step'])" >> gpurun_out/${TAG}.txt || exit 1
done
