#!/bin/bash
# bench probes (--probe-only) of the default build vs an A/B build ($1), interleaved, two rounds
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=$1
for r in 1 2; do
  timeout -k 10 200 python bench.py --probe-only > gpurun_out/pab_base_$r.json 2> gpurun_out/pab_base_$r.err
  MMT_LIB_AB=$AB timeout -k 10 200 python bench.py --probe-only > gpurun_out/pab_ab_$r.json 2> gpurun_out/pab_ab_$r.err
done
