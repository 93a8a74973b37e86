#!/bin/bash
# per-phase roctx ranges of an eager step (no graph, synchronized at each range end: MMT_ROCTX=2)
# + kernel trace -> tools/roctx_summary.py
set -o pipefail
export TMPDIR=/tmp MMT_ROCTX=2
mkdir -p gpurun_out
B=${1:-512}
timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace -d gpurun_out/roctx_b$B -o run --output-format csv -- python bench.py --no-graph --steps 3 --warmup 2 --no-probes --no-cpu-baseline --batch $B > gpurun_out/roctx_b$B.log 2>&1 &&
python tools/roctx_summary.py gpurun_out/roctx_b$B --out gpurun_out/roctx_b${B}_summary.txt
