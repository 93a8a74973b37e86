// Per-workgroup phase timeline of one GEMM launch (PIPE 1 paths: variants 1 and 2), built with -DMMT_GEMM_TRACE:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DMMT_GEMM_TRACE -I include \
//     tools/gemm_trace.cpp -o tools/gemm_trace
//   ./tools/gemm_trace M N K [variant]
// Timestamps are wall_clock64 (100 MHz) after an s_waitcnt(0): start, first tile stored,
// main loop done, epilogue done.
#include "../multi_modal_transformers_tokenmerge_amd/csrc/gemm.hip"
#include "../multi_modal_transformers_tokenmerge_amd/csrc/core.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 18688, N = argc > 2 ? atoi(argv[2]) : 384,
            K = argc > 3 ? atoi(argv[3]) : 384;
  bf16_t *A, *B, *C;
  (void)hipMalloc(&A, sizeof(bf16_t) * M * K);
  (void)hipMalloc(&B, sizeof(bf16_t) * N * K);
  (void)hipMalloc(&C, sizeof(bf16_t) * M * N);
  (void)hipMemset(A, 0x3c, sizeof(bf16_t) * M * K);
  (void)hipMemset(B, 0x3c, sizeof(bf16_t) * N * K);
  mmt_gemm_set_variant(argc > 4 ? atoi(argv[4]) : 1);
  for (int it = 0; it < 3; ++it)
    mmt_gemm(M, N, K, A, 0, K, B, 1, K, C, MMT_OUT_BF16, N, 1, 0, 0, 0, 1, nullptr, nullptr, 0, nullptr);
  (void)hipDeviceSynchronize();
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  std::vector<unsigned long long> tr((size_t)tiles * 5);
  (void)hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_gemm_trace), sizeof(unsigned long long) * 5 * tiles);
  unsigned long long t0 = ~0ull, t3 = 0;
  for (int i = 0; i < tiles; ++i) {
    t0 = std::min(t0, tr[i * 5]);
    t3 = std::max(t3, tr[i * 5 + 3]);
  }
  double load = 0, main_ = 0, epi = 0;
  std::vector<double> starts;
  for (int i = 0; i < tiles; ++i) {
    load += (tr[i * 5 + 1] - tr[i * 5]) * 10e-3;
    main_ += (tr[i * 5 + 2] - tr[i * 5 + 1]) * 10e-3;
    epi += (tr[i * 5 + 3] - tr[i * 5 + 2]) * 10e-3;
    starts.push_back((tr[i * 5] - t0) * 10e-3);
  }
  std::sort(starts.begin(), starts.end());
  printf("M=%d N=%d K=%d tiles=%d span %.2f us | avg per WG: first load %.2f us, main %.2f us, "
         "epilogue %.2f us | start times p0 %.2f p50 %.2f p90 %.2f max %.2f us\n",
         M, N, K, tiles, (t3 - t0) * 10e-3, load / tiles, main_ / tiles, epi / tiles, starts[0],
         starts[tiles / 2], starts[tiles * 9 / 10], starts.back());
  for (int i = 0; i < std::min(tiles, 8); ++i)
    printf("  wg %d se/cu %llx: %.2f %.2f %.2f %.2f\n", i, tr[i * 5 + 4], (tr[i * 5] - t0) * 10e-3,
           (tr[i * 5 + 1] - t0) * 10e-3, (tr[i * 5 + 2] - t0) * 10e-3, (tr[i * 5 + 3] - t0) * 10e-3);
  return 0;
}
