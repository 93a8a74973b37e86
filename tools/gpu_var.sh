set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/var.log
for i in 1 2; do for v in -1 6 7; do
  echo "== v$v" >> gpurun_out/var.log
  MMT_GEMM_VARIANT=$v timeout -k 10 100 python tools/epi_bench.py down dX384 oproj >> gpurun_out/var.log 2>&1 || exit 1
done; done
