#!/bin/bash
# kernel trace of a short bench.py run under an environment (ENVV="VAR=val ..."), kept for
# tools/solo_segments.py / queue analysis: usage ENVV=... tools/gpu_trace_env.sh TAG BATCH
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/tr_$1
export $ENVV
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_$1 -o run -- \
  python3 $R/bench.py --batch $2 --steps 6 --warmup 3 --no-probes --no-cpu-baseline > $R/gpurun_out/tr_$1.log 2>&1
