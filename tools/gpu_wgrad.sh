#!/bin/bash
# weight-gradient products (tools/wgrad_bench.py) on the default build and on an A/B build
# ($1, default libmmt_hip_cb8.so: the combine with 8 slab loads in flight), each under
# rocprofv3 --stats so the GEMM and the combine are timed apart; then the step A/B of the two
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
AB=${1:-multi_modal_transformers_tokenmerge_amd/libmmt_hip_cb8.so}
rm -rf gpurun_out/wg_base gpurun_out/wg_ab
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/wg_base -o wg --output-format csv -- python3 tools/wgrad_bench.py > gpurun_out/wg_base.log 2>&1 &&
MMT_LIB_AB=$AB timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/wg_ab -o wg --output-format csv -- python3 tools/wgrad_bench.py > gpurun_out/wg_ab.log 2>&1 &&
bash tools/gpu_ab_env.sh MMT_LIB_AB "multi_modal_transformers_tokenmerge_amd/libmmt_hip.so $AB" 2
