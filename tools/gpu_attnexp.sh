#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/attnexp
mkdir -p $O
L=multi_modal_transformers_tokenmerge_amd/libmmt_hip.so
for v in a128 a256 a128 a256; do
  cp gpu_exp/lib_$v.so $L &&
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_norm_gpu.py > $O/t_$v.log 2>&1 &&
  timeout -k 10 200 python tools/attn_bench.py > $O/ab_$v.log 2>&1 &&
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit 1
  tail -1 $O/t_$v.log | sed "s/^/$v /"
  grep -v amdgpu $O/ab_$v.log | sed "s/^/$v /"
  tail -1 $O/bench_$v.log | cut -c80-125 | sed "s/^/$v /"
done
cp gpu_exp/lib_a256.so $L
