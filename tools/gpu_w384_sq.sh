#!/bin/bash
# SQ counters of the 384-wide NT kernel on the MLP input-gradient shape (MT 256)
set -o pipefail
export TMPDIR=/tmp MMT_W384_MT=256
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/wsq1 -o run --output-format csv -- python tools/w384_one.py > gpurun_out/wsq1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS --kernel-trace -d gpurun_out/wsq2 -o run --output-format csv -- python tools/w384_one.py > gpurun_out/wsq2.log 2>&1
