#!/bin/bash
# one config's step throughput under environment settings, interleaved:
#   tools/gpu_cfg_ab.sh CONFIG BATCH "VAR=a VAR=b ..." [rounds]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C=$1; B=$2; SETS=$3; R=${4:-1}
for r in $(seq 1 $R); do
  for kv in $SETS; do
    env $kv timeout -k 10 250 python bench.py --config $C --batch $B --no-cpu-baseline --no-probes > gpurun_out/cfgab_${C}_${kv}_$r.log 2>&1 || exit 1
    echo "$C B=$B $kv round $r $(grep -o '"value": [0-9.]*' gpurun_out/cfgab_${C}_${kv}_$r.log)" >> gpurun_out/cfg_ab.txt
  done
done
