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
// The fp8 weight path (BASELINE configs[4], mmt_gemm_fp8) runs the same kernel on e4m3 operands at
// K = 768: a row is again 768 bytes (48 16-B units), the 24 register units hold 12 fragments of
// v_mfma_scale_f32_32x32x64_f8f6f4 (lane (r, h) takes bytes 32h .. 32h+31 of its row's 64-byte
// K-step, the pairing of gemm_fp8_nt_kernel), twice the bf16 FLOPs per chunk at the same cycles.
// Epilogue (XsEpi, gemm_xs.h): fp8 row / channel scales, alpha, bias, relu, counter-RNG dropout,
// in epilogue_w's order, bf16 out. Requires K == 384 (bf16) / 768 (fp8), N % 64 == 0, 16-B aligned
// rows. Rows >= M are read as zeros, never stored.
#include "gemm_xs.h"

#include <algorithm>
#include <type_traits>

using namespace mmt;

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef int v8i __attribute__((ext_vector_type(8)));

constexpr int XS_RB = 768;                         // bytes per X / W row (bf16 K 384, fp8 K 768)
constexpr int XS_ROWS = 256, XS_NC = 64;           // panel rows, chunk columns
constexpr int XS_UNITS16 = XS_RB / 16;             // 48 16-B units per row
constexpr int XS_XR = XS_RB / 32;                  // 24 register units of X per lane
constexpr int XS_SLOT = XS_NC * XS_RB;             // 48 KB per ring slot
constexpr int XS_PIECES = XS_SLOT / 1024 / 8;      // 6 DMA pieces per wave per chunk
// per ring slot, the chunk's 64 bias values (and fp8 channel scales) arrive by LDS-DMA with its
// W rows: two 1-KB pieces (only their first 256 B are read), issued by waves 7 (bias) and 6 (sb)
// fp8 slots: rows padded to 49 units (784 B) instead of the XOR swizzle — unit (r, c) at
// 49 r + c is conflict-free for 16 consecutive rows (49 = 1 mod 16) and every fragment read of a
// lane is one base address + an immediate (the XOR form's 24 per-step addresses spilled the
// fp8 kernel's registers). 49 DMA pieces per slot: wave 0 issues 7, the others 6.
constexpr int XS8_UPR = XS_UNITS16 + 1;            // 49 units per padded row
constexpr int XS8_SLOT = XS_NC * XS8_UPR * 16;     // 50,176 B
constexpr int XS8_PIECES = XS8_SLOT / 1024;        // 49

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
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

#ifndef XS_ABL  // ablation builds (benchmarks only): 1 no W DMA after the prologue, 2 no MFMAs,
#define XS_ABL 0  // 4 no C stores
#endif

// RB (bf16 only): also the relu-bit image of the output (include/mmt_api.h relu_bits layout: bit
// set iff the stored value is > 0), two 16-bit stores per lane per chunk
template <bool F8, bool RB = false>
__global__ __launch_bounds__(512, 1) void gemm_xs_kernel(int M, int N, const char* __restrict__ X,
                                                         int64_t ldxb, const char* __restrict__ W,
                                                         int64_t ldwb, bf16_t* __restrict__ C,
                                                         int64_t ldc, XsEpi e, int n_units) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int SLOT = F8 ? XS8_SLOT : XS_SLOT;
  __shared__ __attribute__((aligned(16))) char ring[3 * SLOT];
  __shared__ __attribute__((aligned(16))) char aux[3][2][1024];  // [slot][bias | sb] of the chunk
  const int lane = threadIdx.x & 63, hh = lane >> 5, lr = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nc = N / XS_NC;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int u0 = (int)((int64_t)n_units * wg / gridDim.x);
  const int u1 = (int)((int64_t)n_units * (wg + 1) / gridDim.x);
  const int nu = u1 - u0;
  if (nu <= 0) return;
  float s_row = 1.f;  // fp8: this lane's row scale in the current panel (loaded with its X)
  const uint32_t key = e.rng ? stream_key(e.rng[0], e.rng[1], e.drop_layer, e.drop_site) : 0u;

  // DMA source offset of this lane in piece p (the slot layout does not depend on the chunk;
  // recomputed per issue: a few VALU ops instead of six registers held across the kernel)
  auto voff = [&](int p) {
    if constexpr (F8) {  // padded rows: unit 48 of a row is padding (loads unit 47, never read)
      const int u = p * 64 + lane;
      const int r = u / XS8_UPR, c = u - r * XS8_UPR;
      return r * (int)ldwb + min(c, XS_UNITS16 - 1) * 16;
    } else {
      const int u = (wave * XS_PIECES + p) * 64 + lane;  // physical unit this lane fills
      const int r = u / XS_UNITS16, pc = u - r * XS_UNITS16;
      const int c = (pc & ~15) | ((pc ^ r) & 15);
      return r * (int)ldwb + c * 16;
    }
  };
  // DMA pieces this wave issues per chunk (bf16: 6; fp8: 7 for wave 0, 6 for the others)
  const int pw = (F8 ? (XS8_PIECES - 1 - wave) / 8 + 1 : XS_PIECES) + (wave == 7 || (F8 && wave == 6) ? 1 : 0);
  auto issue = [&](int j) {  // chunk u0 + j into slot j % 3: pw vm ops per wave
    const int c = (u0 + j) % nc;
    const char* base = W + (int64_t)c * XS_NC * ldwb;
    char* slot = ring + (j % 3) * SLOT;
    // the chunk's bias (wave 7) / fp8 channel scales (wave 6): 64 floats = lanes 0-15 of a piece
    // (a NULL bias reads as zeros: empty buffer range); the rest of the 1-KB piece is not read
    if (wave == 7)
      dma16_asm(e.bias ? (const void*)(e.bias + c * XS_NC) : (const void*)W, e.bias ? XS_NC * 4 : 0,
                aux[j % 3][0], 16 * (lane & 15));
    if (F8 && wave == 6)
      dma16_asm(e.sb + c * XS_NC, XS_NC * 4, aux[j % 3][1], 16 * (lane & 15));
    if constexpr (F8) {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const int p = wave + 8 * k;
        if (p < XS8_PIECES)  // wave-uniform
          dma16_asm(base, (int64_t)XS_NC * ldwb, slot + p * 1024, voff(p));
      }
    } else {
#pragma unroll
      for (int p = 0; p < XS_PIECES; ++p)
        dma16_asm(base, (int64_t)XS_NC * ldwb, slot + (wave * XS_PIECES + p) * 1024, voff(p));
    }
  };
  // per-panel buffer resources: rows past M are out of range (loads read 0, stores are dropped),
  // so every load / store is issued unconditionally and the vm counts below are exact
  auto rsrc = [&](const void* base, int panel, int64_t ldb) {
    const int rows = min(M - panel * XS_ROWS, XS_ROWS);
    return __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(reinterpret_cast<const char*>(base) + (int64_t)panel * XS_ROWS * ldb),
        (short)0, (int)(rows * ldb), 0x00020000);
  };
  // register unit i of this lane: bf16 — fragment i (k-step of 16: 16 B at 32 i + 16 h); fp8 —
  // half i & 1 of fragment i >> 1 (k-step of 64 bytes: 32 B at 64 (i >> 1) + 32 h)
  auto xoff = [&](int i) { return F8 ? 64 * (i >> 1) + 16 * (i & 1) + 32 * hh : 32 * i + 16 * hh; };
  // bf16: 24 fragments of 16 B; fp8: 12 fragments of 32 B held as the 8-register tuples the
  // scaled MFMA takes (assembled from two 16-B pieces would copy 8 registers per MFMA)
  constexpr int XF = F8 ? XS_XR / 2 : XS_XR;
  typedef typename std::conditional<F8, v8i, uint4>::type xfrag_t;
  xfrag_t xq[XF];
  const int xrow = (32 * wave + lr) * (int)ldxb;
  auto ld16 = [&](const __amdgpu_buffer_rsrc_t& rx, int i) {
    return __builtin_amdgcn_raw_buffer_load_b128(rx, xrow + xoff(i), 0, 0);
  };
  auto load_frag = [&](const __amdgpu_buffer_rsrc_t& rx, int f) {  // (F8 ? 2 : 1) vm ops
    if constexpr (F8) {
      const auto a = ld16(rx, 2 * f), b = ld16(rx, 2 * f + 1);
      xq[f] = v8i{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
    } else {
      xq[f] = __builtin_bit_cast(uint4, ld16(rx, f));
    }
  };
  auto load_x = [&](int panel) {  // XS_XR vm ops per wave
    const __amdgpu_buffer_rsrc_t rx = rsrc(X, panel, ldxb);
#pragma unroll
    for (int f = 0; f < XF; ++f) load_frag(rx, f);
  };
  const int coff = (32 * wave + lr) * (int)(ldc * 2) + 16 * hh;

  // epilogue of one 32-column block: lane row m = lr, columns 32 bq + 8 g + 4 hh + i (2 stores);
  // epilogue_w's arithmetic and order. Returns (RB) the positive-value bits, bit 4 g + i.
  auto epilogue = [&](const floatx16& a, int bq, int c, int panel, const __amdgpu_buffer_rsrc_t& rc,
                      const float* cb, const float* csb) {
    const int gr = panel * XS_ROWS + 32 * wave + lr;
    uint32_t pk[4][2];
    uint32_t nib = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = c * XS_NC + 32 * bq + 8 * g + 4 * hh;
      const float4 bb = *reinterpret_cast<const float4*>(cb + 32 * bq + 8 * g + 4 * hh);
      float v[4] = {a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]};
      if constexpr (F8) {
        const float4 sw = *reinterpret_cast<const float4*>(csb + 32 * bq + 8 * g + 4 * hh);
        v[0] = v[0] * s_row * sw.x;
        v[1] = v[1] * s_row * sw.y;
        v[2] = v[2] * s_row * sw.z;
        v[3] = v[3] * s_row * sw.w;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] *= e.alpha;
      v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
      if (e.relu)
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], 0.f);
      if (e.rng) {
        const uint32_t base = (uint32_t)((e.drop_row_offset + gr) * (int64_t)N + col);  // even
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const uint32_t d = pair_draw(key, (base + i) >> 1);
          v[i] = ((d & 0xffffu) < e.keep_thresh16) ? v[i] * e.drop_scale : 0.f;
          v[i + 1] = ((d >> 16) < e.keep_thresh16) ? v[i + 1] * e.drop_scale : 0.f;
        }
      }
      if constexpr (RB)
#pragma unroll
        for (int i = 0; i < 4; ++i) nib |= (v[i] > 0.f ? 1u : 0u) << (4 * g + i);
      pk[g][0] = xs_pk2(v[0], v[1]);
      pk[g][1] = xs_pk2(v[2], v[3]);
    }
#pragma unroll
    for (int g = 0; g < 4; g += 2) {
      const auto x0 = __builtin_amdgcn_permlane32_swap(pk[g][0], pk[g + 1][0], false, false);
      const auto x1 = __builtin_amdgcn_permlane32_swap(pk[g][1], pk[g + 1][1], false, false);
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      const i32x4 d = {(int)x0[0], (int)x1[0], (int)x0[1], (int)x1[1]};
      if (!(XS_ABL & 4))
        __builtin_amdgcn_raw_buffer_store_b128(d, rc, coff + 2 * (c * XS_NC + 32 * bq + 8 * g), 0, 0);
    }
    return gr < M ? nib : 0u;  // (rows past M: no bits, as the 256-wide kernel leaves them)
  };
  // relu-bit image (RB): output (m, n) is bit 8 cb + e of word (g' N/32 + w) 4 + f with
  // g' = (m / 256) 64 + ((m / 64) & 3) 16 + (m & 15), f = (m / 16) & 3 and
  // n = 256 (w / 8) + 128 ((w / 4) & 1) + 8 (w & 3) + 32 cb + e. Chunk c (64 columns) fills bytes
  // cb = bq + 2 (c & 1) of words w = 8 (c / 4) + 4 ((c / 2) & 1) + g, g < 4: one 16-bit half per
  // (row, g), bits e = 4 hh + i from lane (lr, hh). Lane hh stores the halves of g = 2 hh, 2 hh + 1.
  auto store_bits = [&](uint32_t n0, uint32_t n1, int c, const __amdgpu_buffer_rsrc_t& rb) {
    const int rb_row = ((((wave >> 1) * 16 + (lr & 15)) * (N / 32)) * 4 + (wave & 1) * 2 + (lr >> 4)) * 4;
    const uint32_t mine = n0 | (n1 << 16);
    const auto sw = __builtin_amdgcn_permlane32_swap(mine, mine, false, false);
    const uint32_t lo = sw[0], hi = sw[1];  // lane (lr, 0)'s and lane (lr, 1)'s bits in every lane
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int g = 2 * hh + k;
      const uint32_t b0 = ((lo >> (4 * g)) & 15u) | (((hi >> (4 * g)) & 15u) << 4);
      const uint32_t b1 = ((lo >> (16 + 4 * g)) & 15u) | (((hi >> (16 + 4 * g)) & 15u) << 4);
      const int w = 8 * (c >> 2) + 4 * ((c >> 1) & 1) + g;
      __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(b0 | (b1 << 8)), rb,
                                            rb_row + w * 16 + 2 * (c & 1), 0, 0);
    }
  };
  // one chunk: wait + barrier, the ring DMA two chunks ahead, the MFMAs, the epilogue. REFILL
  // (the panel's last chunk when the range continues): each X unit is reloaded with the next
  // panel's as soon as its MFMAs have issued, so the next panel's X streams in under this chunk's
  // MFMAs and epilogue instead of with the chunk loop stopped.
  constexpr int SC = RB ? 6 : 4;  // stores per lane per chunk
  auto chunk = [&](int j, int c, int panel, const __amdgpu_buffer_rsrc_t& rc,
                   const __amdgpu_buffer_rsrc_t& rb, auto refill_tag,
                   const __amdgpu_buffer_rsrc_t& rx_next) {
    constexpr bool REFILL = decltype(refill_tag)::value;
    // chunk j landed: younger than its pieces are the last two chunks' SC stores each and chunk
    // j + 1's pieces (exact: every vm op is unconditional; X loads are drained at each panel
    // start); then publish it. Every wave is then past chunk j - 1's fragment reads, so its slot
    // takes chunk j + 2.
    xs_wait_vm(j < 2 ? 0 : 2 * SC + (j + 1 < nu ? pw : 0));
    asm volatile("s_barrier" ::: "memory");
    if (j + 2 < nu && !(XS_ABL & 1)) issue(j + 2);
    const char* slot = ring + (j % 3) * SLOT;
    floatx16 acc[2];
#pragma unroll
    for (int bq = 0; bq < 2; ++bq)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[bq][r] = 0.f;
    constexpr int STEPS = XF;
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
#pragma unroll
      for (int bq = 0; bq < 2; ++bq) {
        const int r = 32 * bq + lr;
        if constexpr (F8) {
          // logical units 4 s + 2 h and 4 s + 2 h + 1 of padded row r
          const char* wp = slot + r * (XS8_UPR * 16) + 32 * hh + 64 * s;
          const uint4 w0 = *reinterpret_cast<const uint4*>(wp);
          const uint4 w1 = *reinterpret_cast<const uint4*>(wp + 16);
          const v8i wf = {(int)w0.x, (int)w0.y, (int)w0.z, (int)w0.w, (int)w1.x, (int)w1.y, (int)w1.z, (int)w1.w};
          if (!(XS_ABL & 2))
            acc[bq] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf, xq[s], acc[bq], 0, 0, 0, 127, 0, 127);

        } else {
          // logical chunk 2 s + hh of row r
          const bf16x8 wf = *reinterpret_cast<const bf16x8*>(slot + xs_unit(r, 2 * s + hh) * 16);
          if (!(XS_ABL & 2))
            acc[bq] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, __builtin_bit_cast(bf16x8, xq[s]), acc[bq], 0, 0, 0);
        }
      }
      if constexpr (REFILL) load_frag(rx_next, s);
      // fp8: a k-step's fragment reads stay in that k-step (hoisted over all 12 k-steps, the
      // 32-byte W fragments took 96 registers)
      if constexpr (F8) asm volatile("" ::: "memory");
    }
    uint32_t nb[2];
#pragma unroll
    for (int bq = 0; bq < 2; ++bq)
      nb[bq] = epilogue(acc[bq], bq, c, panel, rc, reinterpret_cast<const float*>(aux[j % 3][0]),
                        reinterpret_cast<const float*>(aux[j % 3][1]));
    if constexpr (RB) store_bits(nb[0], nb[1], c, rb);
  };

  issue(0);
  if (nu > 1) issue(1);
  int j = 0;  // chunk counter over the workgroup's range (ring slot j % 3)
  int panel = u0 / nc;
  load_x(panel);
  auto load_sa = [&](int pn) {
    if constexpr (F8) s_row = e.sa[min(pn * XS_ROWS + 32 * wave + lr, M - 1)];
  };
  load_sa(panel);
  for (; j < nu; ++panel) {
    // the panel's X is complete here, by a wait the compiler's vmcnt bookkeeping sees (no X wait
    // then lands inside the chunk loop, where it would also drain the ring DMA)
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0) only (expcnt 7, lgkmcnt 15: no wait)
    const int c_first = u0 + j - panel * nc;
    const int c_end = min(u1 - panel * nc, nc);
    // the range continues into the next panel (fp8: no refill under the last chunk — the
    // second set of live fragments exceeds the 256 registers; the panel start waits instead)
    const bool more = !F8 && !RB && u1 > (panel + 1) * nc;
    const __amdgpu_buffer_rsrc_t rc = rsrc(C, panel, ldc * 2);
    const __amdgpu_buffer_rsrc_t rxn = rsrc(X, more ? panel + 1 : panel, ldxb);
    // the panel's 64 x N/32 relu-bit words (the image has a word row for every row of the last
    // panel, also those past M)
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
        RB ? reinterpret_cast<char*>(e.relu_bits) + (int64_t)panel * N * 32 : reinterpret_cast<char*>(C),
        (short)0, RB ? N * 32 : 0, 0x00020000);
    for (int c = c_first; c < c_end - (more ? 1 : 0); ++c, ++j)
      chunk(j, c, panel, rc, rb, std::false_type{}, rxn);
    if (more) {
      chunk(j, c_end - 1, panel, rc, rb, std::true_type{}, rxn);
      ++j;
    } else if (j < nu) {
      load_x(panel + 1);
    }
    load_sa(panel + 1);  // (drained at the next panel start; never used past the range)
  }
#endif
}

}  // namespace

namespace mmt {

bool xs_shape_ok(int M, int N, int K, bool f8, int64_t lda, int64_t ldb, int64_t ldc, const void* A,
                 const void* B, const void* C, const XsEpi& e) {
  const int esz = f8 ? 1 : 2;
  return M > 0 && K * esz == XS_RB && N > 0 && N % XS_NC == 0 && !e.residual &&
         (lda * esz) % 16 == 0 && (ldb * esz) % 16 == 0 && ldc % 8 == 0 && lda >= K && ldb >= K &&
         ldc >= N && (int64_t)XS_ROWS * std::max(lda * esz, ldc * 2) < 0x7fffffff &&
         (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16 == 0) &&
         (!e.bias || (uintptr_t)e.bias % 16 == 0) && (!f8 || (e.sa && e.sb && (uintptr_t)e.sb % 16 == 0)) &&
         (!e.relu_bits || (!f8 && N % 256 == 0 && (int64_t)N * 32 < 0x7fffffff &&
                           (uintptr_t)e.relu_bits % 16 == 0));
}

int xs_launch(int M, int N, int K, bool f8, const void* X, int64_t lda, const void* W, int64_t ldb,
              void* C, int64_t ldc, int out_f32, const XsEpi& e, hipStream_t stream) {
  MMT_CHECK_ARG(!out_f32 && xs_shape_ok(M, N, K, f8, lda, ldb, ldc, X, W, C, e),
                "gemm_xs: needs %s K, N %% %d == 0, 16-B rows, bf16 out, no residual",
                f8 ? "768-byte" : "384", XS_NC);
  const int panels = (M + XS_ROWS - 1) / XS_ROWS;
  const int n_units = panels * (N / XS_NC);
  int dev = 0, n_cu = 256;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
    n_cu = 256;
  const int grid = std::min(n_units, n_cu);
  const int esz = f8 ? 1 : 2;
  if (f8)
    hipLaunchKernelGGL(gemm_xs_kernel<true>, dim3(grid), dim3(512), 0, stream, M, N, (const char*)X,
                       lda * esz, (const char*)W, ldb * esz, (bf16_t*)C, ldc, e, n_units);
  else if (e.relu_bits)
    hipLaunchKernelGGL((gemm_xs_kernel<false, true>), dim3(grid), dim3(512), 0, stream, M, N,
                       (const char*)X, lda * esz, (const char*)W, ldb * esz, (bf16_t*)C, ldc, e, n_units);
  else
    hipLaunchKernelGGL(gemm_xs_kernel<false>, dim3(grid), dim3(512), 0, stream, M, N, (const char*)X,
                       lda * esz, (const char*)W, ldb * esz, (bf16_t*)C, ldc, e, n_units);
  MMT_CHECK_LAUNCH("gemm_xs");
  return MMT_OK;
}

}  // namespace mmt

extern "C" int mmt_gemm_xs(int M, int N, int K, const void* X, int64_t ldx, const void* W,
                           int64_t ldw, void* C, int64_t ldc, const float* bias,
                           mmt_stream_t stream) {
  MMT_CHECK_ARG(X && W && C && M > 0, "mmt_gemm_xs: bad args");
  XsEpi e;
  e.bias = bias;
  return xs_launch(M, N, K, false, X, ldx, W, ldw, C, ldc, 0, e, as_stream(stream));
}
