#!/bin/bash
# Round-end measurement at the default batch: probe PMC traffic passes (FETCH_SIZE, WRITE_SIZE),
# the full bench line (probes + cpu_baseline) reading that traffic, and a kernel-trace profile of
# the step. Usage: tools/gpu_measure.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02_b512}
mkdir -p gpurun_out
if [ -z "$SKIP_PMC" ]; then  # SKIP_PMC=1: the bench / profile legs only (kernel sources unchanged)
timeout -k 10 200 python bench.py --probe-only > gpurun_out/${TAG}_probes.json 2> gpurun_out/${TAG}_probes.err &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_fetch -o run --output-format csv -- python bench.py --probe-only > gpurun_out/${TAG}_pmc1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_write -o run --output-format csv -- python bench.py --probe-only > gpurun_out/${TAG}_pmc2.log 2>&1 &&
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write --probes gpurun_out/${TAG}_probes.json --out gpurun_out/${TAG}_probe_pmc.json > gpurun_out/${TAG}_pmc3.log 2>&1 &&
cp gpurun_out/${TAG}_probe_pmc.json profiles/ || exit 1
fi
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_benchprof -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/${TAG}_benchprof.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/${TAG}_prof.log 2>&1
