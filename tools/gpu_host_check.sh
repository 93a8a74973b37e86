set -o pipefail
mkdir -p gpurun_out
for B in 128 512; do
  timeout -k 10 250 python bench.py --batch $B --steps 30 --warmup 5 --no-cpu-baseline --no-probes > gpurun_out/host_$B.log 2>&1 || exit 1
  echo "B=$B $(grep -o '"value": [0-9.]*' gpurun_out/host_$B.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/host_$B.log) $(grep -o '"host_ms_per_step_call": [0-9.]*' gpurun_out/host_$B.log)"
done
