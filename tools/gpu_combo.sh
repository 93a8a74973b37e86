set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_var.sh || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 100 --timeout-method thread > gpurun_out/tg.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/ab_new$i.log 2>&1 &&
  MMT_LIB_AB=ab/libmmt_old.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-probes > gpurun_out/ab_old$i.log 2>&1 || exit 1
done
