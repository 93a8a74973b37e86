#!/bin/bash
# Round measurement set: full GPU tests, smoke, bench (with CPU baseline), kernel-trace profile
# of the bench, profile of the probe GEMM alone, and the two PMC passes for its HBM traffic.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/m_tests.log 2>&1 &&
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/m_smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/m_bench.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/m_prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/m_prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/m_probe -o run --output-format csv -- python bench.py --probe-only > gpurun_out/m_probe.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --probe-only > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --probe-only > gpurun_out/pmc_write.log 2>&1
rc=$?
echo "exit $rc" >> gpurun_out/m_tests.log
exit $rc
