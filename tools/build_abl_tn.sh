#!/bin/bash
# ablation builds of the two-stage TN weight-gradient kernel (-DMMT_TN_ABL=N: 1 no DMA, 2 no MFMA,
# 3 no fragment reads after the first k-slice, 4 neither DMA nor reads) linked with the other
# objects into libmmt_hip_tnablN.so (load with MMT_LIB_AB); run after the normal build
set -e
cd "$(dirname "$0")/../multi_modal_transformers_tokenmerge_amd/csrc"
objs=$(ls _obj/*.o | grep -v "/gemm.o$")
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics \
    -ffp-contract=fast -DMMT_TN_ABL=$n -I ../../include -c gemm.hip -o /tmp/gemm_tnabl$n.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../libmmt_hip_tnabl$n.so /tmp/gemm_tnabl$n.o $objs
done
