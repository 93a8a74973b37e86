set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab_t5.txt
timeout -k 10 300 python -u -m pytest tests/test_octo_gpu.py tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_t5_tests.log 2>&1 || exit 1
for b in 128 256 512; do for i in 1 2; do
  timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-probes > gpurun_out/ab_t5_new.log 2>&1 &&
  MMT_LIB_AB=ab/libmmt_old.so timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-probes > gpurun_out/ab_t5_old.log 2>&1 || exit 1
  echo "B=$b new $(grep -o '"value": [0-9.]*' gpurun_out/ab_t5_new.log) old $(grep -o '"value": [0-9.]*' gpurun_out/ab_t5_old.log)" >> gpurun_out/ab_t5.txt
done; done
