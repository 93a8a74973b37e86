#!/bin/bash
# SQ counter passes over the headline dW shape (tools/tn_probe.py --shapes=0): libmmt's TN kernel
# and hipBLASLt's kernel on the same operands, two passes of 8 SQ counters each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
A="tools/tn_probe.py --shapes=0"
rm -rf gpurun_out/tnpmc1 gpurun_out/tnpmc2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d gpurun_out/tnpmc1 -o run --output-format csv -- python $A > gpurun_out/tnpmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES --kernel-trace -d gpurun_out/tnpmc2 -o run --output-format csv -- python $A > gpurun_out/tnpmc2.log 2>&1 &&
for k in gemm_tn_dma16_kernel Cijk_; do echo "== $k"; python tools/pmc_summary.py $k gpurun_out/tnpmc1 gpurun_out/tnpmc2; done > gpurun_out/tn_sq.txt
rm -rf gpurun_out/tnpmc1 gpurun_out/tnpmc2
