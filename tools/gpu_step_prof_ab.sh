#!/bin/bash
# kernel-trace profiles of the step for two builds (libmmt_hip.so vs AB, default libmmt_hip_old.so)
# plus the plain step A/B: per-kernel solo times of short kernels the bench probes do not cover.
#   tools/gpu_step_prof_ab.sh TAG   (per-kernel comparison: tools/kstats_diff.py TAG)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-sprof}
AB=${AB:-multi_modal_transformers_tokenmerge_amd/libmmt_hip_old.so}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_new -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/${TAG}_profnew.log 2>&1 &&
MMT_LIB_AB=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_old -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-probes > gpurun_out/${TAG}_profold.log 2>&1 &&
bash tools/gpu_env_ab.sh ${TAG} "new:" "old:MMT_LIB_AB=$AB"
