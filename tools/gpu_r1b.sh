#!/bin/bash
# smoke + bench with the CPU baseline + kernel-trace profile + two PMC passes on the probe GEMM.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --probe-only > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --probe-only > gpurun_out/pmc_write.log 2>&1
rc=$?
echo "exit $rc" >> gpurun_out/smoke.log
exit $rc
