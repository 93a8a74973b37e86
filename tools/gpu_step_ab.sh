#!/bin/bash
# step A/B with the bench probes (roofline.kernels) and the T5 encoder probe: libmmt_hip.so vs a
# second build (AB=path, default libmmt_hip_old.so), interleaved; optional pytest files first.
#   TESTS="tests/test_gemm_gpu.py" tools/gpu_step_ab.sh TAG
set -o pipefail
TAG=${1:-ab}
AB=${AB:-multi_modal_transformers_tokenmerge_amd/libmmt_hip_old.so}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread $TESTS > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
fi
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --no-cpu-baseline > gpurun_out/${TAG}_new$r.log 2>&1 || exit 1
  MMT_LIB_AB=$AB timeout -k 10 300 python -u bench.py --steps 30 --warmup 8 --no-cpu-baseline > gpurun_out/${TAG}_old$r.log 2>&1 || exit 1
done
if [ -n "$T5" ]; then
  timeout -k 10 200 python -u tools/t5_encoder_probe.py > gpurun_out/${TAG}_t5new.log 2>&1 || exit 1
  MMT_LIB_AB=$AB timeout -k 10 200 python -u tools/t5_encoder_probe.py > gpurun_out/${TAG}_t5old.log 2>&1 || exit 1
fi
