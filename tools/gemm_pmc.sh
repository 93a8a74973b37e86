#!/bin/bash
# GEMM micro-benchmark (+ hipBLASLt reference) and one SQ counter pass over it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_bench.py --torch > gpurun_out/gemm_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/gemm_pmc -o run --output-format csv -- python tools/gemm_bench.py > gpurun_out/gemm_pmc.log 2>&1
