#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread \
  tests/test_heads_gpu.py tests/test_sampler_gpu.py tests/test_c_abi.py > gpurun_out/r1e_tests.log 2>&1
