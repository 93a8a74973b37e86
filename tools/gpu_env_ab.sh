#!/bin/bash
# step A/B over environments (each "NAME:VAR=val,VAR2=val"; "base" entries may set MMT_LIB_AB),
# interleaved rounds, bench probes on; optional TESTS first. Summary: tools/ab_summary.py TAG
#   TESTS=... tools/gpu_env_ab.sh TAG "new:" "res0:MMT_NTW_RES=0" "old:MMT_LIB_AB=...so"
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread $TESTS > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
fi
for r in 1 2; do
  for v in "$@"; do
    n=${v%%:*}; e=${v#*:}
    env ${e//,/ } timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --no-cpu-baseline > gpurun_out/${TAG}_$n$r.log 2>&1 || exit 1
  done
done
