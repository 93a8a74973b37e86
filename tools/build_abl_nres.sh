#!/bin/bash
# ablation builds of the residual-stream kernel (-DMMT_NRES_ABL=N: 1 no W DMA, 2 no A DMA, 3 no
# MFMA, 4 no epilogue loads / stores, 5 no DMA) linked with the other objects into
# libmmt_hip_nresablN.so (load with MMT_LIB_AB); run after the normal build
set -e
cd "$(dirname "$0")/../multi_modal_transformers_tokenmerge_amd/csrc"
objs=$(ls _obj/*.o | grep -v "/gemm.o$")
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics \
    -ffp-contract=fast -DMMT_NRES_ABL=$n -I ../../include -c gemm.hip -o /tmp/gemm_nresabl$n.o &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../libmmt_hip_nresabl$n.so /tmp/gemm_nresabl$n.o $objs
done
