#!/bin/bash
# mmt_gemm kernel choice per shape: default dispatch vs forced nt256 tile widths (variants 5/6/7)
# at B = 512 (tools/gemm_bench.py)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default 6 7 5; do
  if [ "$v" = default ]; then a=""; else a="--variant=$v"; fi
  timeout -k 10 240 python tools/gemm_bench.py --b=512 $a > gpurun_out/gemm_v$v.log 2>&1 || exit 1
done
