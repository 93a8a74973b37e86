#!/bin/bash
# CPU sanitizer builds (test infrastructure, never shipped or run on a GPU box):
#  * the ToMe oracle oracle/tome_ref.c + tests/asan/tome_ref_driver.c with gcc ASan + UBSan;
#  * the host half of libmmt_hip's ToMe / pruning / core dispatch (core.hip, tome.hip, prune.hip
#    compiled with the host half instrumented; their device code is built but never launched) + tests/asan/abi_host_driver.cpp with hipcc,
#    the address sanitizer on the host side only.
# Outputs go to $1 (default /tmp/mmt_asan), outside the repository.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(cd "$HERE/../.." && pwd)"
OUT="${1:-/tmp/mmt_asan}"
mkdir -p "$OUT"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
gcc -O1 -g -std=c11 -ffp-contract=off -fno-omit-frame-pointer -fsanitize=address,undefined \
  -fno-sanitize-recover=all "$ROOT/oracle/tome_ref.c" "$HERE/tome_ref_driver.c" -lm \
  -o "$OUT/tome_ref_asan"
HOSTFLAGS=(-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address
           -Xarch_host -fno-omit-frame-pointer -ffp-contract=off -Wno-pass-failed -w -I "$ROOT/include")
for f in core tome prune; do
  "$HIPCC" "${HOSTFLAGS[@]}" -c "$ROOT/multi_modal_transformers_tokenmerge_amd/csrc/$f.hip" \
    -o "$OUT/$f.o" &
done
wait
CLANGXX="${CLANGXX:-/opt/rocm/lib/llvm/bin/clang++}"
"$CLANGXX" -O1 -g -std=c++17 -fno-omit-frame-pointer -fsanitize=address -I "$ROOT/include" \
  -c "$HERE/abi_host_driver.cpp" -o "$OUT/abi_host_driver.o"
"$CLANGXX" -O1 -g -std=c++17 -fsanitize=address -c "$HERE/det_units_stub.cpp" -o "$OUT/det_units_stub.o"
"$HIPCC" --hip-link -Xarch_host -fsanitize=address "$OUT/abi_host_driver.o" "$OUT/core.o" \
  "$OUT/tome.o" "$OUT/prune.o" "$OUT/det_units_stub.o" -o "$OUT/abi_host_asan"
