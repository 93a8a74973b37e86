#!/bin/bash
# HBM / L2 counters of the 384-wide NT kernel on the MLP input-gradient shape
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
export MMT_W384_MT=256
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/wpmc1 -o run --output-format csv -- python tools/w384_one.py > gpurun_out/wpmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/wpmc2 -o run --output-format csv -- python tools/w384_one.py > gpurun_out/wpmc2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d gpurun_out/wpmc3 -o run --output-format csv -- python tools/w384_one.py > gpurun_out/wpmc3.log 2>&1
