#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_tome_gpu.py tests/test_octo_gpu.py -q -x > gpurun_out/tome_t.log 2>&1 &&
timeout -k 10 200 python tools/tome_bench.py > gpurun_out/tome_b.log 2>&1
