// LDS-DMA fill-rate lab (round 5): how fast can one CU fill LDS with buffer_load_dwordx4 ... lds
// for the access patterns of the library's LDS-staged GEMMs, and what caps the ~32 GB/s per CU
// their mainloops reach (gemm_tn_dma_kernel, gemm_glds_nt_kernel)? No compute: only the DMA, the
// waits and the barriers of each structure.
//   hipcc -O3 --offload-arch=gfx950 -o tools/dma_lab tools/dma_lab.hip && tools/dma_lab
// Source: a 2 GB bf16 matrix of 3072-B rows (the MLP Dense_0 dY layout) — each workgroup streams
// its own K range of 64-row steps, reading `cols` bytes of every row at column offset `c0` (768 B
// = one 384-column tile of the TN kernel) — or, with l2 = 1, every workgroup the same 64 rows.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void dma16(const void* base, long bytes, void* lds, int voffset) {
  const unsigned long b = (unsigned long)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
  r[1] = __builtin_amdgcn_readfirstlane((int)((unsigned)(b >> 32) & 0xffffu));
  r[2] = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7ffffff0 ? bytes : 0x7ffffff0));
  r[3] = 0x00020000;
  const unsigned l = __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long)((__attribute__((address_space(3))) char*)lds));
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voffset), "s"(r), "s"(l) : "m0", "memory");
}

// MODE 0: two stages, every wave issues its pieces of step s + 1 right after the barrier,
//         then vmcnt(0) + barrier (the TN kernel's structure)
// MODE 1: NST-stage ring, pieces of step s + NST - 1 issued after the barrier, counted vmcnt
// MODE 2: no barriers: each wave streams its own pieces through its own ring slots, keeping
//         `ahead` steps in flight (counted vmcnt), the fastest a wave can feed its share
template <int MODE, int NW, int NST, int COLS>
__global__ __launch_bounds__(NW * 64, 1) void dma_kernel(const char* __restrict__ src, long ld,
                                                         long rows_total, int c0,
                                                         int steps, int l2, unsigned* sink) {
  constexpr int cols = COLS;
  constexpr int PER = 64 * COLS / 1024 / NW;       // pieces per wave per step
  static_assert(PER >= 1 && PER <= 16 && (NST - 2) * PER < 64, "pieces");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int step_bytes = 64 * cols;                 // one 64-row step
  const int pieces = step_bytes / 1024;             // 1-KB pieces per step
  const int per_wave = PER;
  (void)pieces;
  // 768-B slices: 4 consecutive workgroups read the 4 slices of the same rows (as the TN kernel's
  // 4 M-tiles of one K-split), so whole 3-KB rows are fetched
  const int grp = cols == 768 ? blockIdx.x >> 2 : blockIdx.x;
  if (cols == 768) c0 = (blockIdx.x & 3) * 768;
  const long row0 = l2 ? 0 : (long)grp * steps * 64 % (rows_total - steps * 64);
  const int chunks = cols / 16;
  int voff[16];
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int e = (wave * per_wave + (p < per_wave ? p : 0)) * 64 + lane;
    voff[p] = (e / chunks) * (int)ld + (e % chunks) * 16;
  }
  auto issue = [&](int s, int slot) {
    const long r = l2 ? 0 : row0 + (long)s * 64;
    const char* base = src + r * ld + c0;
    char* dst = smem + slot * step_bytes + wave * per_wave * 1024;
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (p < per_wave) dma16(base, (rows_total - r) * ld - c0, dst + p * 1024, voff[p]);
  };
  if (MODE == 0) {
    issue(0, 0);
    for (int s = 0; s < steps; ++s) {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      if (s + 1 < steps) issue(s + 1, (s + 1) & 1);
    }
  } else if (MODE == 1) {
    for (int q = 0; q < NST - 1; ++q) issue(q, q);
    for (int s = 0; s < steps; ++s) {
      // younger than step s: steps s + 1 .. s + NST - 2 (PER pieces each)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER * (NST - 2)) : "memory");
      asm volatile("s_barrier" ::: "memory");
      if (s + NST - 1 < steps) issue(s + NST - 1, (s + NST - 1) % NST);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    for (int q = 0; q < NST - 1; ++q) issue(q, q);
    for (int s = 0; s < steps; ++s) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER * (NST - 2)) : "memory");
      if (s + NST - 1 < steps) issue(s + NST - 1, (s + NST - 1) % NST);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = ((unsigned*)smem)[lane];
}

// The TN weight-gradient kernel's own fill pattern (gemm_tn_dma16_kernel at the MLP Dense_0 dW
// shape, M = 1536, N = 384, K = 141,312, split 32): workgroup wi -> (split z, tile t) after the
// XCD remap, A = 64 k-rows x 768 B of dY (3072-B rows), B = 64 k-rows x 384 B of X (768-B rows),
// KS k-rows per step (64: 9 pieces per wave; 32: 4.5), NST stages, DMA NST - 1 steps ahead
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}
template <int KS, int NST, bool BAR>
__global__ __launch_bounds__(512, 1) void tn_dma_kernel(const char* __restrict__ A, const char* __restrict__ B,
                                                        int K, int k_chunk, unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int A_BYTES = KS * 768, STAGE = KS * (768 + 384);
  constexpr int PT = STAGE / 1024;       // pieces per step (72 or 36)
  constexpr int PW = (PT + 7) / 8;       // per wave (9 or 5; the last waves fewer at 36)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wi = xcd_remap(blockIdx.x, gridDim.x);
  const int z = wi / 8, t = wi % 8, tm = t / 2, tn = t % 2;
  const int m0 = tm * 384, n0 = tn * 192;
  const int kbeg = z * k_chunk, nk = k_chunk / KS;
  int voff[PW], isA[PW], lds_off[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int j = wave * PW + i;            // wave-contiguous pieces
    const int jj = j < PT ? j : PT - 1;
    const int byte = jj * 1024;
    isA[i] = byte < A_BYTES;
    if (isA[i]) {
      const int e = jj * 64 + lane, row = e / 48, c = e % 48;
      voff[i] = row * 3072 + c * 16;
    } else {
      const int e = (jj - A_BYTES / 1024) * 64 + lane, row = e / 24, c = e % 24;
      voff[i] = row * 768 + c * 16;
    }
    lds_off[i] = jj * 1024;
  }
  const long bytesA = (long)K * 3072, bytesB = (long)K * 768;
  auto issue = [&](int s, int slot) {
    const long k0 = kbeg + (long)s * KS;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      if (wave * PW + i >= PT) break;
      if (isA[i]) dma16(A + k0 * 3072 + m0 * 2, bytesA - k0 * 3072 - m0 * 2, smem + slot * STAGE + lds_off[i], voff[i]);
      else dma16(B + k0 * 768 + n0 * 2, bytesB - k0 * 768 - n0 * 2, smem + slot * STAGE + lds_off[i], voff[i]);
    }
  };
  for (int q = 0; q < NST - 1; ++q) issue(q, q);
  for (int s = 0; s < nk; ++s) {
    if constexpr (NST == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW * (NST - 2)) : "memory");
    if (BAR) asm volatile("s_barrier" ::: "memory");
    if (s + NST - 1 < nk) issue(s + NST - 1, (s + NST - 1) % NST);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = ((unsigned*)smem)[lane];
}
template <int KS, int NST, bool BAR>
void run_tn(const char* name, const char* A, const char* B, unsigned* sink) {
  const int K = 141312, split = 32, k_chunk = K / split;
  const int lds = NST * KS * (768 + 384);
  auto k = tn_dma_kernel<KS, NST, BAR>;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k, dim3(256), dim3(512), lds, 0, A, B, K, k_chunk, sink);
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k, dim3(256), dim3(512), lds, 0, A, B, K, k_chunk, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps;
  const double fills = 256.0 * k_chunk * (768 + 384), uniq = (double)K * (3072 + 768);
  printf("%-44s %8.1f us  fills %6.1f GB/s per CU, unique %5.2f TB/s\n", name, us, fills / us / 1e3 / 256,
         uniq / us / 1e6);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

template <int MODE, int NW, int NST, int cols>
void run(const char* name, const char* src, long ld, long rows, int c0, int steps, int l2,
         int grid, unsigned* sink) {
  const int lds = NST * 64 * cols;
  if (lds > 163840) {
    printf("%-44s skipped (LDS %d B)\n", name, lds);
    return;
  }
  auto k = dma_kernel<MODE, NW, NST, cols>;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, 0, src, ld, rows, c0, steps, l2, sink);
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, 0, src, ld, rows, c0, steps, l2, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / reps;
  const double bytes = (double)grid * steps * 64 * cols;
  printf("%-44s %8.1f us  %6.2f TB/s chip  %6.1f GB/s per CU\n", name, us, bytes / us / 1e6,
         bytes / us / 1e3 / grid);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main() {
  const long ld = 3072;                      // bytes per row (1536 bf16)
  const long rows = 2L * 1024 * 1024 * 1024 / ld;
  char* src;
  unsigned* sink;
  CHECK(hipMalloc(&src, rows * ld));
  CHECK(hipMalloc(&sink, 4096 * sizeof(unsigned)));
  CHECK(hipMemset(src, 1, rows * ld));
  const int grid = 256, steps = 64;
  {
    char *A, *B;
    CHECK(hipMalloc(&A, 141312L * 3072));
    CHECK(hipMalloc(&B, 141312L * 768));
    CHECK(hipMemset(A, 1, 141312L * 3072));
    CHECK(hipMemset(B, 1, 141312L * 768));
    printf("== the TN kernel's fill pattern alone (MLP Dense_0 dW, split 32, 256 workgroups)\n");
    run_tn<64, 2, true>("TN fills: 2 x 64-row stages, barrier", A, B, sink);
    run_tn<64, 2, false>("TN fills: 2 x 64-row stages, no barrier", A, B, sink);
    run_tn<32, 4, true>("TN fills: 4 x 32-row ring, barrier", A, B, sink);
    run_tn<32, 4, false>("TN fills: 4 x 32-row ring, no barrier", A, B, sink);
    run_tn<16, 8, true>("TN fills: 8 x 16-row ring, barrier", A, B, sink);
    CHECK(hipFree(A));
    CHECK(hipFree(B));
  }
  for (int l2 = 0; l2 < 2; ++l2) {
    printf("== source: %s\n", l2 ? "the same 64 rows for every workgroup (L2)" : "HBM, own rows per workgroup");
    // 768-B row slices (the TN kernel's A tile), 48 KB per step
    run<0, 8, 2, 768>("2-stage, 8 waves, 768 B x 64 rows", src, ld, rows, 768, steps, l2, grid, sink);
    run<0, 4, 2, 768>("2-stage, 4 waves, 768 B x 64 rows", src, ld, rows, 768, steps, l2, grid, sink);
    run<1, 8, 3, 768>("3-stage ring, 8 waves, 768 B x 64", src, ld, rows, 768, steps, l2, grid, sink);
    run<2, 8, 3, 768>("no barrier, 8 waves, 3 slots, 768 B x 64", src, ld, rows, 768, steps, l2, grid, sink);
    run<2, 4, 3, 768>("no barrier, 4 waves, 3 slots, 768 B x 64", src, ld, rows, 768, steps, l2, grid, sink);
    // full 3-KB rows... as 2 x 1536-B halves (96 KB per step: 1 stage + a partial would not fit)
    run<0, 8, 2, 1024>("2-stage, 8 waves, 1024 B x 64 rows", src, ld, rows, 0, steps, l2, grid, sink);
    run<2, 8, 2, 1024>("no barrier, 8 waves, 2 slots, 1024 B x 64", src, ld, rows, 0, steps, l2, grid, sink);
    run<0, 8, 2, 512>("2-stage, 8 waves, 512 B x 64 rows", src, ld, rows, 0, steps, l2, grid, sink);
    run<1, 8, 4, 512>("4-stage ring, 8 waves, 512 B x 64", src, ld, rows, 0, steps, l2, grid, sink);
    run<2, 8, 4, 512>("no barrier, 8 waves, 4 slots, 512 B x 64", src, ld, rows, 0, steps, l2, grid, sink);
    run<2, 4, 4, 512>("no barrier, 4 waves, 4 slots, 512 B x 64", src, ld, rows, 0, steps, l2, grid, sink);
  }
  CHECK(hipFree(src));
  CHECK(hipFree(sink));
  return 0;
}
