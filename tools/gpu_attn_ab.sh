#!/bin/bash
# attention A/B: tools/attn_bench.py under two environments, interleaved (ENV_A / ENV_B: "VAR=val ...")
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  echo "== A ($ENV_A) round $r"; env $ENV_A timeout -k 10 200 python -u tools/attn_bench.py --b=512 --L=292,228,164 2>&1 | grep octo || exit 1
  echo "== B ($ENV_B) round $r"; env $ENV_B timeout -k 10 200 python -u tools/attn_bench.py --b=512 --L=292,228,164 2>&1 | grep octo || exit 1
done
