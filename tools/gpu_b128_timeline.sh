#!/bin/bash
# Small-batch step timelines: kernel trace of bench.py --batch B, per-queue
# busy time, idle gaps and the serial-only kernels (tools/timeline.py) and the kernel stats.
# usage: bash tools/gpu_b128_timeline.sh "128 512" [tag]   (env passes through, e.g. MMT_TN_KERNEL)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${2:-}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for B in ${1:-128 512}; do
  rm -rf $R/gpurun_out/tl$B$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tl$B$TAG -o run -- \
    python3 $R/bench.py --batch $B --steps 20 --warmup 5 --no-probes --no-cpu-baseline > $R/gpurun_out/tl$B$TAG.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/tl$B$TAG -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/timeline.py $f 5 --gaps > $R/gpurun_out/timeline_b$B$TAG.txt || exit 1
  g=$(find $R/gpurun_out/tl$B$TAG -name "*kernel_stats.csv" | head -1)
  python3 $R/tools/kstats.py $g 40 > $R/gpurun_out/kstats_b$B$TAG.txt 2>&1 || true
  rm -f $f
done
