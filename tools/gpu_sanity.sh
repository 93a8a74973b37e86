#!/bin/bash
# Quick sanity pass on a fresh box: GPU tests, smoke, default bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s_smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/s_bench.log 2>&1
