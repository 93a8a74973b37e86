#!/bin/bash
# persistent attention forward: bit-identity / tolerance tests, then forward timing of the
# persistent kernel (two-pass and one-pass) vs the resident one
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attn_norm_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/attn_pers_test.log 2>&1 || exit 1
for cfg in "MMT_ATTN_ONEPASS=1" "MMT_ATTN_ONEPASS=0" "MMT_ATTN_PERS=1"; do
  echo "== $cfg" >> gpurun_out/attn_pers_bench.txt
  env $cfg timeout -k 10 200 python tools/attn_bench.py --b=512 --L=292,212,116 >> gpurun_out/attn_pers_bench.txt 2>&1 || exit 1
done
