#!/bin/bash
# ablation builds of gemm.hip (-DMMT_W384_ABL=N: 1 no B DMA, 2 no DMA, 3 no MFMA) linked with the
# other objects into libmmt_hip_ablN.so (load with MMT_LIB_AB); run after the normal build
set -e
cd "$(dirname "$0")/../multi_modal_transformers_tokenmerge_amd/csrc"
objs=$(ls _obj/*.o | grep -v "/gemm.o$")
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics \
    -ffp-contract=fast -DMMT_W384_ABL=$n -I ../../include -c gemm.hip -o /tmp/gemm_abl$n.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../libmmt_hip_abl$n.so /tmp/gemm_abl$n.o $objs
done
