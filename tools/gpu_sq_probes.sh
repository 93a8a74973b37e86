#!/bin/bash
# SQ counter passes over the bench probes (bench.py --probe-only: every probe kernel launched alone
# at the step's block-0 shapes): where the waves of the step's heaviest kernels spend their time.
# Usage: tools/gpu_sq_probes.sh TAG  (summaries by tools/pmc_summary.py)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r06_sq}
mkdir -p gpurun_out
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --kernel-trace -d gpurun_out/${TAG}_1 -o run --output-format csv -- python bench.py --probe-only > gpurun_out/${TAG}_1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES --kernel-trace -d gpurun_out/${TAG}_2 -o run --output-format csv -- python bench.py --probe-only > gpurun_out/${TAG}_2.log 2>&1
