#!/bin/bash
# counter passes over tools/attn_bench.py at B=512, L=292 (resident attention kernels): two SQ
# passes and the HBM fetch / write passes
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
A="tools/attn_bench.py --b=512 --L=292"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d gpurun_out/apmc1 -o run --output-format csv -- python $A > gpurun_out/apmc1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES --kernel-trace -d gpurun_out/apmc2 -o run --output-format csv -- python $A > gpurun_out/apmc2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/apmc3 -o run --output-format csv -- python $A > gpurun_out/apmc3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/apmc4 -o run --output-format csv -- python $A > gpurun_out/apmc4.log 2>&1
