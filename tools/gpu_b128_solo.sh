#!/bin/bash
# B = 128 step trace kept for tools/solo_segments.py (where one queue runs alone)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for B in ${1:-128}; do
  rm -rf $R/gpurun_out/solo$B
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/solo$B -o run -- \
    python3 $R/bench.py --batch $B --steps 6 --warmup 3 --no-probes --no-cpu-baseline > $R/gpurun_out/solo$B.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/solo$B -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/solo_segments.py $f 15 > $R/gpurun_out/solo_b$B.txt || exit 1
done
