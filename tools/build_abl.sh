#!/bin/bash
# ablation builds of attention.hip (-DMMT_RES_ABL=N) linked with the other objects into
# libmmt_hip_ablN.so (load with MMT_LIB_AB); run after the normal build
set -e
cd "$(dirname "$0")/../multi_modal_transformers_tokenmerge_amd/csrc"
objs=$(ls _obj/*.o | grep -v attention)
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -munsafe-fp-atomics \
    -ffp-contract=fast -fno-honor-nans -mno-amdgpu-ieee -DMMT_RES_ABL=$n -I ../../include -c attention.hip -o /tmp/attn_abl$n.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../libmmt_hip_abl$n.so /tmp/attn_abl$n.o $objs
done
