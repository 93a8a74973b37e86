// Per-tile timeline of the persistent nt256 GEMM (gemm_nt256_kernel), built with -DMMT_GEMM_TRACE:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DMMT_GEMM_TRACE -I include tools/nt_trace.cpp -o tools/nt_trace
//   ./tools/nt_trace M N K [variant 5|6|7] [out_f32]
// wall_clock64 (100 MHz) stamps by thread 0: K-step 0 landed, main loop done, epilogue issued.
#include "../multi_modal_transformers_tokenmerge_amd/csrc/gemm.hip"
#include "../multi_modal_transformers_tokenmerge_amd/csrc/core.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace mmt {  // core.hip's workspace query links against tome.hip; not needed here
int64_t tome_match_workspace(int64_t, int64_t, int64_t) { return 0; }
}  // namespace mmt

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 70656, N = argc > 2 ? atoi(argv[2]) : 1536,
            K = argc > 3 ? atoi(argv[3]) : 384;
  const int var = argc > 4 ? atoi(argv[4]) : 5, f32 = argc > 5 ? atoi(argv[5]) : 0;
  bf16_t *A, *B;
  void* C;
  (void)hipMalloc(&A, sizeof(bf16_t) * M * K);
  (void)hipMalloc(&B, sizeof(bf16_t) * N * K);
  (void)hipMalloc(&C, 4ull * M * N);
  (void)hipMemset(A, 0x3c, sizeof(bf16_t) * M * K);
  (void)hipMemset(B, 0x3c, sizeof(bf16_t) * N * K);
  mmt_gemm_set_variant(var);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int it = 0; it < 5; ++it) {
    if (it == 4) (void)hipEventRecord(e0, nullptr);
    mmt_gemm(M, N, K, A, 0, K, B, 1, K, C, f32 ? MMT_OUT_F32 : MMT_OUT_BF16, N, 1, 0, 0, 0, 1,
             nullptr, nullptr, 0, nullptr);
  }
  (void)hipEventRecord(e1, nullptr);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const int bn = var == 5 ? 256 : var == 6 ? 192 : 128;
  const int tiles = ((M + 255) / 256) * (N / bn), grid = std::min(tiles, 256);
  std::vector<unsigned long long> tr((size_t)1024 * 16 * 3);
  (void)hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_nt_trace), tr.size() * 8);
  auto T = [&](int w, int i, int s) { return tr[((size_t)w * 16 + i) * 3 + s]; };
  unsigned long long t0 = ~0ull, tend = 0;
  for (int w = 0; w < grid; ++w) t0 = std::min(t0, T(w, 0, 0));
  double main_ = 0, epi = 0, gap = 0;
  int nm = 0, ng = 0;
  for (int w = 0; w < grid; ++w) {
    const int xcd = w & 7, q = grid >> 3, r = grid & 7;  // host copy of xcd_remap
    const int f = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (w >> 3);
    const int mine = (tiles - f + grid - 1) / grid;
    for (int i = 0; i < std::min(mine, 16); ++i) {
      main_ += (T(w, i, 1) - T(w, i, 0)) * 10e-3;
      epi += (T(w, i, 2) - T(w, i, 1)) * 10e-3;
      ++nm;
      if (i + 1 < std::min(mine, 16)) {
        gap += (T(w, i + 1, 0) - T(w, i, 2)) * 10e-3;
        ++ng;
      }
      tend = std::max(tend, T(w, i, 2));
    }
  }
  printf("M=%d N=%d K=%d BN=%d f32=%d tiles=%d grid=%d  kernel %.1f us  trace span %.1f us | per tile: "
         "main %.2f us, epilogue issue %.2f us, epilogue->next K-step0 %.2f us\n",
         M, N, K, bn, f32, tiles, grid, ms * 1e3, (tend - t0) * 10e-3, main_ / nm, epi / nm, gap / std::max(ng, 1));
  for (int w = 0; w < 4; ++w) {
    printf("  wg %d:", w);
    for (int i = 0; i < 8; ++i)
      printf(" [%.1f %.1f %.1f]", (T(w, i, 0) - t0) * 10e-3, (T(w, i, 1) - t0) * 10e-3, (T(w, i, 2) - t0) * 10e-3);
    printf("\n");
  }
  {
    std::vector<unsigned long long> ck((size_t)1024 * 4);
    (void)hipMemcpyFromSymbol(ck.data(), HIP_SYMBOL(g_nt_clk), ck.size() * 8);
    std::vector<double> f;
    for (int w = 0; w < grid; ++w) {
      const double dc = (double)(ck[w * 4 + 2] - ck[w * 4]), dr = (double)(ck[w * 4 + 3] - ck[w * 4 + 1]);
      if (dr > 0) f.push_back(dc / dr * 100.0);  // MHz (memrealtime = 100 MHz)
    }
    std::sort(f.begin(), f.end());
    if (!f.empty()) printf("  in-kernel clock MHz: min %.0f median %.0f max %.0f\n", f[0], f[f.size() / 2], f.back());
  }
  std::vector<unsigned long long> st((size_t)1024 * 2 * 16 * 5);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_nt_step), st.size() * 8);
  for (int w = 0; w < 2; ++w)
    for (int h = 0; h < 2; ++h) {
      printf("  wg %d wave %d steps [issue wait barrier compute end] us:\n", w, 4 * h);
      for (int k = 0; k < 14; ++k) {
        const unsigned long long* p = &st[(((size_t)w * 2 + h) * 16 + k) * 5];
        printf("    s%2d: %7.2f %7.2f %7.2f %7.2f %7.2f\n", k, (p[0] - t0) * 10e-3, (p[1] - t0) * 10e-3,
               (p[2] - t0) * 10e-3, (p[3] - t0) * 10e-3, (p[4] - t0) * 10e-3);
      }
    }
  return 0;
}
