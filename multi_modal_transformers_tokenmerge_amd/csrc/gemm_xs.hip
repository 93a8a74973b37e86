// Activation-stationary NT GEMM for the short-K products of the OCTO-small block (K = D = 384):
// C[M][N] = epi(X[M][K] . W[N][K]^T). The QKV projection (N = 1152) and the MLP up-projection
// (N = 1536) read a 115 MB activation X against a 0.9-1.2 MB weight: nt256's 256 x 256 tiles fetch
// each X row panel once per column tile (6 times at N = 1536; 2.05x algorithmic reads measured
// with L2 catching the rest) and stage both operands through LDS per K-step.
// Here a workgroup holds a 256-row panel of X in REGISTERS for the whole N sweep:
//  * 8 waves x 32 rows; a wave's 32 x 384 slice is 24 MFMA B-operand fragments (96 VGPRs), read
//    once from HBM (global_load_dwordx4, 16 B of a row per lane);
//  * W streams through a 3-slot LDS ring in 64-column chunks (64 x 384 bf16 = 48 KB, LDS-DMA by all
//    8 waves, issued two chunks ahead, one barrier per chunk); W stays L2-resident;
//  * per chunk each wave runs 2 x 24 v_mfma_f32_32x32x16_bf16 (W fragment = A operand, so the
//    accumulator is C^T: lane = output row, 16 columns in runs of 4) and stores its 32 x 64 tile
//    through the v_permlane32_swap pairing (16-B stores, 32 contiguous bytes per row per half);
//  * persistent grid, chunk-granular balance: the (panel, chunk) units in panel-major order are
//    cut into equal contiguous ranges, one per workgroup (every CU within one unit of the mean),
//    and a workgroup reloads X only when its range crosses into a new panel.
// Per 64-column chunk a CU computes 2.1 MFLOP from 48 KB of W (LDS-DMA) and 32 KB of C stores.
// Requires K == 384, N % 64 == 0, 16-B aligned rows. Rows >= M are read as zeros, never stored.
#include "common.h"

#include <type_traits>

using namespace mmt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

constexpr int XS_K = 384, XS_KS = XS_K / 16;      // 24 MFMA k-steps
constexpr int XS_ROWS = 256, XS_NC = 64;           // panel rows, chunk columns
constexpr int XS_UNITS16 = XS_K / 8;               // 48 16-B units per W row
constexpr int XS_SLOT = XS_NC * XS_K * 2;          // 48 KB per ring slot
constexpr int XS_PIECES = XS_SLOT / 1024 / 8;      // 6 DMA pieces per wave per chunk
constexpr int XS_MAXN = 1536;                      // bias columns staged in LDS

__device__ __forceinline__ uint32_t xs_pk2(float a, float b) {
  const float2v v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}

// physical 16-B unit of (row r, logical 16-B chunk c) in a slot: the low 4 bits of c XOR r, so the
// fragment reads (16 consecutive rows at one chunk per 16-lane group) hit 16 distinct bank groups
__host__ __device__ __forceinline__ int xs_unit(int r, int c) {
  return r * XS_UNITS16 + ((c & ~15) | ((c ^ r) & 15));
}

// vmcnt(n) for the counts the chunk loop needs (immediates)
__device__ __forceinline__ void xs_wait_vm(int n) {
  switch (n) {
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

#ifndef XS_ABL  // ablation builds (benchmarks only): 1 no W DMA after the prologue, 2 no MFMAs,
#define XS_ABL 0  // 4 no C stores
#endif

template <int EP>  // EP 0: bf16 C (+ bias when given)
__global__ __launch_bounds__(512, 1) void gemm_xs_kernel(int M, int N, const bf16_t* __restrict__ X,
                                                         int64_t ldx, const bf16_t* __restrict__ W,
                                                         int64_t ldw, bf16_t* __restrict__ C,
                                                         int64_t ldc, const float* __restrict__ bias,
                                                         int n_units) {
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ __attribute__((aligned(16))) char ring[3 * XS_SLOT];
  __shared__ __attribute__((aligned(16))) float s_bias[XS_MAXN];
  const int lane = threadIdx.x & 63, hh = lane >> 5, lr = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nc = N / XS_NC;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int u0 = (int)((int64_t)n_units * wg / gridDim.x);
  const int u1 = (int)((int64_t)n_units * (wg + 1) / gridDim.x);
  const int nu = u1 - u0;
  if (nu <= 0) return;
  for (int i = threadIdx.x; i < N; i += 512) s_bias[i] = bias ? bias[i] : 0.f;
  __syncthreads();

  // DMA source offsets of this wave's pieces (fixed: the slot layout does not depend on the chunk)
  int voff[XS_PIECES];
#pragma unroll
  for (int p = 0; p < XS_PIECES; ++p) {
    const int u = (wave * XS_PIECES + p) * 64 + lane;  // physical unit this lane fills
    const int r = u / XS_UNITS16, pc = u - r * XS_UNITS16;
    const int c = (pc & ~15) | ((pc ^ r) & 15);
    voff[p] = r * (int)(ldw * 2) + c * 16;
  }
  auto issue = [&](int j) {  // chunk u0 + j into slot j % 3: XS_PIECES vm ops per wave
    const int c = (u0 + j) % nc;
    const bf16_t* base = W + (int64_t)c * XS_NC * ldw;
    char* slot = ring + (j % 3) * XS_SLOT;
#pragma unroll
    for (int p = 0; p < XS_PIECES; ++p)
      dma16_asm(base, (int64_t)XS_NC * ldw * 2, slot + (wave * XS_PIECES + p) * 1024, voff[p]);
  };
  // per-panel buffer resources: rows past M are out of range (loads read 0, stores are dropped),
  // so every load / store is issued unconditionally and the vm counts below are exact
  auto rsrc = [&](const bf16_t* base, int panel, int64_t ld) {
    const int rows = min(M - panel * XS_ROWS, XS_ROWS);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(base + (int64_t)panel * XS_ROWS * ld),
                                             (short)0, (int)(rows * ld * 2), 0x00020000);
  };
  bf16x8 xf[XS_KS];
  const int xoff = (32 * wave + lr) * (int)(ldx * 2) + 16 * hh;
  auto load_x = [&](int panel) {  // XS_KS vm ops per wave
    const __amdgpu_buffer_rsrc_t rx = rsrc(X, panel, ldx);
#pragma unroll
    for (int s = 0; s < XS_KS; ++s)
      xf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rx, xoff + 32 * s, 0, 0));
  };
  const int coff = (32 * wave + lr) * (int)(ldc * 2) + 16 * hh;

  // epilogue of one 32-column block: lane row m = lr, columns 32 bq + 8 g + 4 hh + i (2 stores)
  auto epilogue = [&](const floatx16& a, int bq, int c, const __amdgpu_buffer_rsrc_t& rc) {
    const float* bp = s_bias + c * XS_NC + 32 * bq + 4 * hh;
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      const float4 q0 = *reinterpret_cast<const float4*>(bp + 8 * g);
      const float4 q1 = *reinterpret_cast<const float4*>(bp + 8 * g + 8);
      const uint32_t a0 = xs_pk2(a[4 * g] + q0.x, a[4 * g + 1] + q0.y);
      const uint32_t a1 = xs_pk2(a[4 * g + 2] + q0.z, a[4 * g + 3] + q0.w);
      const uint32_t b0 = xs_pk2(a[4 * g + 4] + q1.x, a[4 * g + 5] + q1.y);
      const uint32_t b1 = xs_pk2(a[4 * g + 6] + q1.z, a[4 * g + 7] + q1.w);
      const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      const i32x4 d = {(int)x0[0], (int)x1[0], (int)x0[1], (int)x1[1]};
      if (!(XS_ABL & 4))
        __builtin_amdgcn_raw_buffer_store_b128(d, rc, coff + 2 * (c * XS_NC + 32 * bq + 8 * g), 0, 0);
    }
  };
  // one chunk: wait + barrier, the ring DMA two chunks ahead, 2 x 24 MFMAs, the epilogue. REFILL
  // (the panel's last chunk when the range continues): each X fragment is reloaded with the next
  // panel's as soon as its two MFMAs have issued, so the next panel's X streams in under this
  // chunk's MFMAs and epilogue instead of with the chunk loop stopped.
  auto chunk = [&](int j, int c, const __amdgpu_buffer_rsrc_t& rc, auto refill_tag,
                   const __amdgpu_buffer_rsrc_t& rx_next) {
    constexpr bool REFILL = decltype(refill_tag)::value;
    // chunk j landed: younger than its pieces are the last two chunks' 4 stores each and chunk
    // j + 1's pieces (exact: every vm op is unconditional; X loads are drained at each panel
    // start); then publish it. Every wave is then past chunk j - 1's fragment reads, so its slot
    // takes chunk j + 2.
    xs_wait_vm(j < 2 ? 0 : 8 + (j + 1 < nu ? XS_PIECES : 0));
    asm volatile("s_barrier" ::: "memory");
    if (j + 2 < nu && !(XS_ABL & 1)) issue(j + 2);
    const char* slot = ring + (j % 3) * XS_SLOT;
    floatx16 acc[2];
#pragma unroll
    for (int bq = 0; bq < 2; ++bq)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[bq][r] = 0.f;
#pragma unroll
    for (int s = 0; s < XS_KS; ++s) {
      // logical chunk 2 s + hh of row r: unit r * 48 + g + ((2 s & 15) + hh) ^ (r & 15)
      const int g = (2 * s) & ~15, cs = (2 * s) & 15;
#pragma unroll
      for (int bq = 0; bq < 2; ++bq) {
        const int r = 32 * bq + lr;
        const int off = (r * XS_UNITS16 + g + ((cs + hh) ^ (r & 15))) * 16;
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(slot + off);
        if (!(XS_ABL & 2)) acc[bq] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, xf[s], acc[bq], 0, 0, 0);
      }
      if constexpr (REFILL)
        xf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rx_next, xoff + 32 * s, 0, 0));
    }
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) epilogue(acc[bq], bq, c, rc);
  };

  issue(0);
  if (nu > 1) issue(1);
  int j = 0;  // chunk counter over the workgroup's range (ring slot j % 3)
  int panel = u0 / nc;
  load_x(panel);
  for (; j < nu; ++panel) {
    // the panel's X is complete here, by a wait the compiler's vmcnt bookkeeping sees (no X wait
    // then lands inside the chunk loop, where it would also drain the ring DMA)
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0) only (expcnt 7, lgkmcnt 15: no wait)
    const int c_first = u0 + j - panel * nc;
    const int c_end = min(u1 - panel * nc, nc);
    const bool more = u1 > (panel + 1) * nc;  // the range continues into the next panel
    const __amdgpu_buffer_rsrc_t rc = rsrc(C, panel, ldc);
    const __amdgpu_buffer_rsrc_t rxn = rsrc(X, more ? panel + 1 : panel, ldx);
    for (int c = c_first; c < c_end - (more ? 1 : 0); ++c, ++j) chunk(j, c, rc, std::false_type{}, rxn);
    if (more) {
      chunk(j, c_end - 1, rc, std::true_type{}, rxn);
      ++j;
    }
  }
#endif
}

}  // namespace

extern "C" int mmt_gemm_xs(int M, int N, int K, const void* X, int64_t ldx, const void* W,
                           int64_t ldw, void* C, int64_t ldc, const float* bias,
                           mmt_stream_t stream) {
  MMT_CHECK_ARG(X && W && C && M > 0, "mmt_gemm_xs: bad args");
  MMT_CHECK_ARG(K == XS_K && N % XS_NC == 0 && N > 0 && N <= XS_MAXN, "mmt_gemm_xs: needs K == %d, N %% %d == 0, N <= %d", XS_K, XS_NC, XS_MAXN);
  MMT_CHECK_ARG((int64_t)XS_ROWS * std::max(ldx, ldc) * 2 < 0x7fffffff, "mmt_gemm_xs: row stride too large");
  MMT_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0 && ldc % 8 == 0 && ldx >= K && ldw >= K && ldc >= N,
                "mmt_gemm_xs: strides (16-B rows)");
  MMT_CHECK_ARG(((uintptr_t)X | (uintptr_t)W | (uintptr_t)C) % 16 == 0 && (!bias || (uintptr_t)bias % 16 == 0),
                "mmt_gemm_xs: 16-B alignment");
  const int panels = (M + XS_ROWS - 1) / XS_ROWS;
  const int n_units = panels * (N / XS_NC);
  int dev = 0, n_cu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = std::min(n_units, n_cu > 0 ? n_cu : 256);
  hipLaunchKernelGGL(gemm_xs_kernel<0>, dim3(grid), dim3(512), 0, as_stream(stream), M, N,
                     (const bf16_t*)X, ldx, (const bf16_t*)W, ldw, (bf16_t*)C, ldc, bias, n_units);
  MMT_CHECK_LAUNCH("mmt_gemm_xs");
  return MMT_OK;
}
