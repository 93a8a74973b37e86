#!/bin/bash
# same-box A/B of the in-tree library against ab/libmmt_old.so (MMT_LIB_AB), alternating runs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_epi.log
for i in 1 2 3; do
  echo "== new $i" >> gpurun_out/ab_epi.log
  timeout -k 10 100 python tools/epi_bench.py "$@" >> gpurun_out/ab_epi.log 2>&1 || exit 1
  echo "== old $i" >> gpurun_out/ab_epi.log
  MMT_LIB_AB=ab/libmmt_old.so timeout -k 10 100 python tools/epi_bench.py "$@" >> gpurun_out/ab_epi.log 2>&1 || exit 1
done
