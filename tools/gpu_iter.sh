set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_nt256_gpu.py tests/test_octo_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1 &&
timeout -k 10 200 python tools/epi_bench.py > gpurun_out/r_epi2.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r_bench2.log 2>&1
