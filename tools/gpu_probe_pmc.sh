#!/bin/bash
# SQ counters (MFMA busy, waits, LDS bank conflicts) of every bench probe kernel, one pass
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d gpurun_out/probe_sq -o run --output-format csv -- python bench.py --probe-only > gpurun_out/probe_sq.log 2>&1
