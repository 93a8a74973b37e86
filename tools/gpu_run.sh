#!/bin/bash
# One GPU box session: each step under its own time limit, chained so a failure stops the run.
# usage: bash tools/gpu_run.sh <step> [<step> ...]; steps below write gpurun_out/<step>.log
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for step in "$@"; do
  case "$step" in
    golden_dump) timeout -k 10 240 python -u tools/golden_diag.py dump small_tome16_2blk && \
                 timeout -k 10 180 python -u tools/golden_diag.py dump ref_octo_base && \
                 du -sh gpurun_out/* ;;
    tn_ring_test) timeout -k 10 240 $T tests/test_gemm_gpu.py -k "tn_" ;;
    tn_probe) timeout -k 10 300 python -u tools/tn_probe.py --variants=${TN_VARIANTS:-10,13} ;;
    tn_probe_lib) timeout -k 10 300 python -u tools/tn_probe.py ;;
    new_tests) timeout -k 10 400 $T tests/test_deterministic_gpu.py tests/test_attn_norm_gpu.py \
                 tests/test_t5_stem_gpu.py ;;
    multiset) timeout -k 10 400 $T tests/test_octo_gpu.py -k "multiset" ;;
    attn_bias) timeout -k 10 300 python -u tools/attn_bias.py ;;
    parity_exact) timeout -k 10 900 python -u tools/parity_exact.py --seeds=8 ;;
    dma_lab) timeout -k 10 120 tools/dma_lab ;;
    tome_tests) timeout -k 10 400 $T tests/test_tome_gpu.py ;;
    tome_bench) timeout -k 10 300 python -u tools/tome_bench.py ;;
    attn_tests) timeout -k 10 400 $T tests/test_attn_norm_gpu.py -k "attention or resident" ;;
    attn_stamps) MMT_LIB_AB=multi_modal_transformers_tokenmerge_amd/libmmt_hip_abl9.so timeout -k 10 200 python -u tools/attn_stamps.py ;;
    attn_bench) timeout -k 10 300 python -u tools/attn_bench.py --b=512 --L=292,228 ;;
    heads) timeout -k 10 300 $T tests/test_heads_gpu.py ;;
    golden) timeout -k 10 240 $T -s tests/test_golden_step_gpu.py ;;
    gpu_all) timeout -k 10 900 $T -m gpu tests ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) timeout -k 10 600 python -u bench.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac > "gpurun_out/$step.log" 2>&1
  rc=$?
  echo "step $step rc=$rc"
  tail -n 4 "gpurun_out/$step.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
