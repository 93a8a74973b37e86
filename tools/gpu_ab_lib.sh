#!/bin/bash
# tests touching the change, then same-box bench A/B of the in-tree library vs ab/libmmt_old.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_attn_norm_gpu.py tests/test_tome_gpu.py tests/test_octo_gpu.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/abl_t.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/abl_new$i.log 2>&1 &&
  MMT_LIB_AB=ab/libmmt_old.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/abl_old$i.log 2>&1 || exit 1
done
