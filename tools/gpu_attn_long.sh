#!/bin/bash
# attention at the OCTO-base lengths (L = 1064 / 788 / 532, H = 12, B = 32): backward workgroup
# size A/B, then configs[3] with the current defaults
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for nt in 128 256; do
  MMT_ATTN_BWD_NT=$nt timeout -k 10 200 python tools/attn_bench.py --b=32 --h=12 --L=1064,788,532 > gpurun_out/attn_long_bnt$nt.log 2>&1 || exit 1
done
timeout -k 10 400 python bench.py --config octo-base-2cam --batch 32 --no-cpu-baseline --steps 30 --warmup 5 --no-probes > gpurun_out/base2cam.log 2>&1
