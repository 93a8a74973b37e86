set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_base_configs.sh; echo "base rc=$?" > gpurun_out/batch2_rc.txt
timeout -k 10 900 python -u tools/noise_sources.py --seeds=6 > gpurun_out/noise.log 2>&1; echo "noise rc=$?" >> gpurun_out/batch2_rc.txt
