#!/bin/bash
# round-4 checkpoint: golden-fixture and deterministic-mode tests (printed reports), the whole GPU
# suite + smoke, attention bench, bench line, deterministic-mode step-time A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_golden_step_gpu.py tests/test_deterministic_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/golden.log 2>&1
bash tools/gpu_all.sh
timeout -k 10 200 python tools/attn_bench.py --b=512 --L=292,212,116 > gpurun_out/attn_bench_r04.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04_bench2.log 2>&1 &&
bash tools/gpu_ab_env.sh MMT_DETERMINISTIC "0 1" 2
