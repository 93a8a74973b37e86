#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wexp
mkdir -p $O
L=multi_modal_transformers_tokenmerge_amd/libmmt_hip.so
for v in w192 w256 w192 w256; do
  cp gpu_exp/lib_$v.so $L &&
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$v.log 2>&1 || exit 1
  tail -1 $O/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['roofline']['avg_launch_us'])"
done
cp gpu_exp/lib_w256.so $L
