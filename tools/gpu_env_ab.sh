#!/bin/bash
# bench A/B of an environment knob: tools/gpu_env_ab.sh "VAR=a" "VAR=b" (alternating, 2 rounds) + trace of the first
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/eab_a$i.log 2>&1 &&
  env $2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/eab_b$i.log 2>&1 || exit 1
done
export $1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/eab_prof -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/eab_prof.log 2>&1
