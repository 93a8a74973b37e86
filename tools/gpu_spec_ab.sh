set -o pipefail
mkdir -p gpurun_out /tmp/fb
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_norm_gpu.py > gpurun_out/spec_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/attn_fwd_bits.py /tmp/fb/new.pt > gpurun_out/spec_bits.log 2>&1 || exit 1
MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_base.so timeout -k 10 120 python tools/attn_fwd_bits.py /tmp/fb/base.pt >> gpurun_out/spec_bits.log 2>&1 || exit 1
python tools/attn_fwd_bits.py --compare /tmp/fb/new.pt /tmp/fb/base.pt >> gpurun_out/spec_bits.log 2>&1 || exit 1
bash tools/gpu_attn_libs.sh spec default base
