#!/bin/bash
# bench A/B of a Python-side change (MMT_AB=0/1 is read by the code under test) + step trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  MMT_AB=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/pab_new$i.log 2>&1 &&
  MMT_AB=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/pab_old$i.log 2>&1 || exit 1
done
MMT_AB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pab_prof -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/pab_prof.log 2>&1
