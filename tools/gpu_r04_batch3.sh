#!/bin/bash
# configs[4] bench (fixed probes) + fp8 A/B, kernel stats of both OCTO-base configs, the full-depth
# free-running parity test at the tightened bar
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--batch 32 --no-cpu-baseline"
timeout -k 10 400 python bench.py --config octo-base-hires-tome32 $B --steps 30 --warmup 5 > gpurun_out/hires.log 2>&1; echo "hires $?" > gpurun_out/batch3_rc.txt
timeout -k 10 400 python bench.py --config octo-base-hires-tome32 $B --steps 30 --warmup 5 --no-probes --set fp8=0 > gpurun_out/hires_bf16.log 2>&1; echo "hires_bf16 $?" >> gpurun_out/batch3_rc.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base2cam -o run --output-format csv -- python bench.py --config octo-base-2cam $B --steps 5 --warmup 2 --no-probes > gpurun_out/prof_base2cam.log 2>&1; echo "prof2cam $?" >> gpurun_out/batch3_rc.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hires -o run --output-format csv -- python bench.py --config octo-base-hires-tome32 $B --steps 5 --warmup 2 --no-probes > gpurun_out/prof_hires.log 2>&1; echo "profhires $?" >> gpurun_out/batch3_rc.txt
timeout -k 10 600 python -u -m pytest tests/test_octo_gpu.py -k "free_running_full_depth" -x -q -s --timeout 500 --timeout-method thread > gpurun_out/freerun.log 2>&1; echo "freerun $?" >> gpurun_out/batch3_rc.txt
