#!/bin/bash
# Round measurements: PMC traffic of the probe GEMM (two separate passes), the bench line (with
# the CPU baseline), rocprofv3 kernel-trace summaries of the bench and of the probe GEMM.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/m
O=gpurun_out/m
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python bench.py --probe-only > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python bench.py --probe-only > $O/pmc_write.log 2>&1 &&
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write --shape 70656 1536 384 --out profiles/r01_nt256w_gemm_pmc.json > $O/pmc.log 2>&1 &&
cp profiles/r01_nt256w_gemm_pmc.json $O/ &&
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_probe -o run --output-format csv -- python bench.py --probe-only > $O/prof_probe.log 2>&1
