#!/bin/bash
# every BASELINE config on one GPU (bench.py --config NAME --batch B), one line each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/configs.log
for cb in ${CONFIGS:-octo-tiny:512 octo-small:512 octo-small-tome16:512 octo-small-prune16:512 octo-base-2cam:32 octo-base-2cam-tome16:32 octo-base-hires-tome32:32 octo-small-tome16:256}; do
  c=${cb%%:*}; b=${cb##*:}
  timeout -k 10 250 python bench.py --config $c --batch $b --steps 30 --warmup 5 --no-cpu-baseline --no-probes > gpurun_out/cfg_${c}_$b.log 2>&1 || exit 1
  echo "$c B=$b $(grep -o '"value": [0-9.]*, "unit": "samples/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/cfg_${c}_$b.log) $(grep -o '"model_tflops_per_s": [0-9.]*' gpurun_out/cfg_${c}_$b.log)" >> gpurun_out/configs.log
done
