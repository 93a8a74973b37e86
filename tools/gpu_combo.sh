set -o pipefail
mkdir -p gpurun_out
for f in 1 0; do for b in 1 0; do
echo "fwd=$f bwd=$b" >> gpurun_out/combo.log
MMT_ATTN_RES=$f MMT_ATTN_RES_BWD=$b timeout -k 10 200 python -u -m pytest "tests/test_octo_gpu.py::test_e2e_free_running" -q --timeout 120 --timeout-method thread >> gpurun_out/combo.log 2>&1
done; done
exit 0
