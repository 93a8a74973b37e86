// bf16 MFMA GEMM with fused epilogues for gfx950 — the Dense / DenseGeneral layers of the hot
// path (Flax Dense in attention.py:32-37 MLPBlock, SelfAttention QKV/out projections,
// image_tokenizer.py stem convolution-as-GEMM and output Dense, diffusion.py heads, T5 layers).
//
//   C = epilogue( op(A) . op(B) )      op(A): M x K,  op(B): K x N,  fp32 accumulation
//   transA = 0: A stored [M][K] (K contiguous)   transA = 1: A stored [K][M] (M contiguous)
//   transB = 0: B stored [K][N] (N contiguous)   transB = 1: B stored [N][K] (weights W[N][K])
//
// Tile 128 x 128 x 64, 256 threads = 4 waves (2 x 2), each wave a 64 x 64 block of
// v_mfma_f32_32x32x16_bf16. K-contiguous operand tiles are read with ds_read_b128 along k;
// M/N-contiguous tiles (the transposed operands of the backward GEMMs) are staged as they come
// from HBM and read with the gfx950 transpose read ds_read_b64_tr_b16 — no transpose pass in HBM.
// Register-staged double buffer (global loads of tile k+1 issued before the MFMAs of tile k).
// Workgroups are remapped so the tiles sharing an A row-panel run on one XCD (shared L2).
// Epilogue straight from registers: the MFMA operands are swapped so the accumulator holds C^T
// and every lane owns runs of 4 consecutive columns of one row (8-16 B vector bias / gate /
// residual loads and C stores, no LDS round trip).
// Split-K writes fp32 partial slabs (plain stores) reduced by a second kernel — no atomics.
#include "common.h"
#include "gemm_xs.h"

using namespace mmt;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#ifdef MMT_GEMM_TRACE  // tools/gemm_trace.cpp: per-workgroup phase timestamps (wave 0)
__device__ unsigned long long g_gemm_trace[1 << 16][5];
#define GEMM_TRACE(i)                                                                          \
  do {                                                                                         \
    __builtin_amdgcn_s_waitcnt(0);                                                             \
    if (threadIdx.x == 0 && blockIdx.x < (1 << 16)) {                                          \
      g_gemm_trace[blockIdx.x][i] = wall_clock64();                                            \
      if ((i) == 0) g_gemm_trace[blockIdx.x][4] = __smid();                                    \
    }                                                                                          \
  } while (0)
// nt256: per workgroup, per tile (up to 16): K-step 0 landed, main loop done, epilogue issued
__device__ unsigned long long g_nt_trace[1024][16][3];
#define NT_TRACE(ti, slot)                                                                     \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && (ti) < 16)                                    \
      g_nt_trace[blockIdx.x][ti][slot] = wall_clock64();                                       \
  } while (0)
// nt256 in-kernel clock: s_memtime / s_memrealtime at the first K-step and after the last epilogue
__device__ unsigned long long g_nt_clk[1024][4];
#define NT_CLK(slot)                                                                           \
  do {                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 1024) {                                               \
      g_nt_clk[blockIdx.x][2 * (slot)] = __builtin_amdgcn_s_memtime();                         \
      g_nt_clk[blockIdx.x][2 * (slot) + 1] = __builtin_amdgcn_s_memrealtime();                 \
    }                                                                                          \
  } while (0)
// nt256 per-step timeline of wave 0 and wave 4: after DMA issue, after vmcnt wait, after barrier,
// after compute, after the closing barrier (steps 0..15)
__device__ unsigned long long g_nt_step[1024][2][16][5];
#define NT_STEP(st_, slot)                                                                     \
  do {                                                                                         \
    if ((threadIdx.x & 255) == 0 && blockIdx.x < 1024 && (st_) < 16)                           \
      g_nt_step[blockIdx.x][threadIdx.x >> 8][st_][slot] = wall_clock64();                     \
  } while (0)
#else
#define NT_CLK(slot) \
  do {               \
  } while (0)
#define NT_STEP(st_, slot) \
  do {                     \
  } while (0)
#define GEMM_TRACE(i) \
  do {                \
  } while (0)
#define NT_TRACE(ti, slot) \
  do {                     \
  } while (0)
#endif

namespace {

constexpr int BM = 128, BN = 128;
constexpr int NTHREADS = 256;
constexpr int MC_STRIDE = BM + 8;   // M/N-contiguous tile [BK][136] bf16 (272 B rows)
// LDS geometry per K-step depth BKT (64 or 128)
template <int BKT>
struct Geom {
  static constexpr int KCS = BKT + 8;                      // K-contiguous tile [128][BKT+8]
  static constexpr int TILE = 128 * KCS > BKT * MC_STRIDE ? 128 * KCS : BKT * MC_STRIDE;
  static constexpr int Q = 128 * BKT / 8 / NTHREADS;       // 16-B chunks per thread per operand
};

// tuning knob: 0 = PIPE 0 / BK 64, 1 = PIPE 1 / BK 64, 2 = PIPE 1 / BK 128, 3 = 256 x 192 tiles,
// 4 = direct-to-LDS NT kernel; other = automatic (see mmt_gemm)
int g_variant = -1;

struct Epi {
  const float* bias;
  int act;
  uint32_t drop_layer, drop_site, keep_thresh16;
  float drop_scale;
  const uint32_t* rng;
  int64_t drop_row_offset;
  const bf16_t* gate;
  int64_t ld_gate;
  float gate_scale;
  const void* residual;
  int res_f32;
  int64_t ld_res;
  float alpha, beta;
  float* colsum;  // nt256 only: per-256-row-panel column sums of the stored (bf16) C, or null
  uint32_t* relu_bits;         // nt256 BN 256 only: 1 bit per output, set iff stored bf16 > 0
  const uint32_t* gate_bits;   // nt256 BN 256 only: the gate in that 1-bit form
  const uint32_t* keep_bits;   // nt256 relu_bits launches only: dropout keeps in that layout
};

// global -> registers for one 128 x 64 (K-contig) or 64 x 128 (MN-contig) operand tile.
// Branch-free: every chunk loads from an address clamped into range (needs the contiguous
// extent to be a multiple of 8, checked by mmt_gemm); store_tile zeroes the out-of-range chunks
// when it writes LDS. Keeping the mask out of the load lets the compiler count vmcnt waits (a
// predicated load forces vmcnt(0)) and leaves the loads in flight until the store.
// Operand tile of R rows (M or N) x BKT (K) held in LDS either K-contiguous [R][BKT+8] or
// M/N-contiguous [BKT][R+8]; NT threads move it in 16-B chunks, Q = R*BKT/8/NT per thread.
template <bool KCONTIG, int BKT, int R>
__device__ __forceinline__ void chunk_of(int c, int r0, int k0, int& row, int& kk) {
  if (KCONTIG) {  // [row][k]: BKT/8 chunks of 8 per row
    row = r0 + c / (BKT / 8);
    kk = k0 + (c % (BKT / 8)) * 8;
  } else {        // [k][row]: R/8 chunks of 8 per k-row
    kk = k0 + c / (R / 8);
    row = r0 + (c % (R / 8)) * 8;
  }
}

template <bool KCONTIG, int BKT, int R, int NT>
__device__ __forceinline__ void load_tile(const bf16_t* __restrict__ P, int64_t ld, int rows_lim,
                                          int k_lim, int r0, int k0, uint4 (&reg)[R * BKT / 8 / NT]) {
#pragma unroll
  for (int q = 0; q < R * BKT / 8 / NT; ++q) {
    int row, kk;
    chunk_of<KCONTIG, BKT, R>(threadIdx.x + q * NT, r0, k0, row, kk);
    const bf16_t* p = KCONTIG ? P + (int64_t)min(row, rows_lim - 1) * ld + min(kk, k_lim - 8)
                              : P + (int64_t)min(kk, k_lim - 1) * ld + min(row, rows_lim - 8);
    reg[q] = *reinterpret_cast<const uint4*>(p);
  }
}

template <bool KCONTIG, int BKT, int R, int NT>
__device__ __forceinline__ void store_tile(bf16_t* __restrict__ S, const uint4 (&reg)[R * BKT / 8 / NT],
                                           int rows_lim, int k_lim, int r0, int k0) {
#pragma unroll
  for (int q = 0; q < R * BKT / 8 / NT; ++q) {
    const int c = threadIdx.x + q * NT;
    int row, kk;
    chunk_of<KCONTIG, BKT, R>(c, r0, k0, row, kk);
    const uint32_t m = (row < rows_lim && kk < k_lim) ? 0xffffffffu : 0u;
    const int off = KCONTIG ? (c / (BKT / 8)) * (BKT + 8) + (c % (BKT / 8)) * 8
                            : (c / (R / 8)) * (R + 8) + (c % (R / 8)) * 8;
    *reinterpret_cast<uint4*>(S + off) =
        make_uint4(reg[q].x & m, reg[q].y & m, reg[q].z & m, reg[q].w & m);
  }
}

__device__ __forceinline__ short4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)((__attribute__((address_space(3))) void*)p));
}

// MFMA 32x32x16 operand fragment: lane (r = lane&31, h = lane>>5) holds X[r][k = 8h + j].
template <bool KCONTIG, int KCS, int MCS>
__device__ __forceinline__ bf16x8 load_frag(const bf16_t* S, int rbase, int ks, int lane) {
  if (KCONTIG) {
    const bf16_t* p = S + (rbase + (lane & 31)) * KCS + ks * 16 + 8 * (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const int i = lane & 15, q = i >> 2, p4 = i & 3, g = lane >> 4, h = lane >> 5;
    const int col = rbase + 16 * (g & 1) + 4 * p4;
    const int k1 = ks * 16 + 8 * h + q;
    const short4v v1 = tr_read(S + k1 * MCS + col);
    const short4v v2 = tr_read(S + (k1 + 4) * MCS + col);
    short __attribute__((ext_vector_type(8))) v = {v1[0], v1[1], v1[2], v1[3],
                                                   v2[0], v2[1], v2[2], v2[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// W consecutive elements (W = 4 or 8, 8*W/... byte aligned) -> fp32
template <int W>
__device__ __forceinline__ void ldw(const bf16_t* p, float* f) {
  uint32_t w[W / 2];
  if constexpr (W == 8) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    w[0] = u.x; w[1] = u.y;
  }
#pragma unroll
  for (int q = 0; q < W / 2; ++q) {
    f[2 * q] = __uint_as_float(w[q] << 16);
    f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
template <int W>
__device__ __forceinline__ void ldw(const float* p, float* f) {
#pragma unroll
  for (int q = 0; q < W / 4; ++q) {
    const float4 a = *reinterpret_cast<const float4*>(p + 4 * q);
    f[4 * q] = a.x; f[4 * q + 1] = a.y; f[4 * q + 2] = a.z; f[4 * q + 3] = a.w;
  }
}

// Epilogue on W consecutive columns (gc .. gc+W-1, gc even) of output row gr, in place on v[W]:
// alpha, bias, relu, gate, counter-RNG dropout (pairs of 16-bit draws), residual.
template <int W>
__device__ __forceinline__ void epilogue_w(const Epi& epi, uint32_t key, int N, int gr, int gc,
                                           float* v) {
#pragma unroll
  for (int e = 0; e < W; ++e) v[e] *= epi.alpha;
  if (epi.bias) {
    float bb[W];
    ldw<W>(epi.bias + gc, bb);
#pragma unroll
    for (int e = 0; e < W; ++e) v[e] += bb[e];
  }
  if (epi.act == MMT_ACT_RELU)
#pragma unroll
    for (int e = 0; e < W; ++e) v[e] = fmaxf(v[e], 0.f);
  if (epi.gate) {
    float g[W];
    ldw<W>(epi.gate + (int64_t)gr * epi.ld_gate + gc, g);
#pragma unroll
    for (int e = 0; e < W; ++e) v[e] *= (g[e] > 0.f) ? epi.gate_scale : 0.f;
  }
  if (epi.rng) {
    const uint32_t base = (uint32_t)((epi.drop_row_offset + gr) * (int64_t)N + gc);  // even
#pragma unroll
    for (int e = 0; e < W; e += 2) {
      const uint32_t d = pair_draw(key, (base + e) >> 1);
      v[e] = ((d & 0xffffu) < epi.keep_thresh16) ? v[e] * epi.drop_scale : 0.f;
      v[e + 1] = ((d >> 16) < epi.keep_thresh16) ? v[e + 1] * epi.drop_scale : 0.f;
    }
  }
  if (epi.residual) {
    float rr[W];
    const int64_t ro = (int64_t)gr * epi.ld_res + gc;
    if (epi.res_f32) ldw<W>(reinterpret_cast<const float*>(epi.residual) + ro, rr);
    else ldw<W>(reinterpret_cast<const bf16_t*>(epi.residual) + ro, rr);
#pragma unroll
    for (int e = 0; e < W; ++e) v[e] += rr[e];
  }
}

// Store W columns: bf16 (OUT 0) or fp32 with C = v + beta * C (OUT 1, or 2 = plain fp32 slab).
template <int OUT, int W>
__device__ __forceinline__ void store_w(void* Cv, int64_t off, float beta, const float* v) {
  if (OUT == 0) {
    uint32_t w[W / 2];
#pragma unroll
    for (int q = 0; q < W / 2; ++q) w[q] = (uint32_t)f2bf(v[2 * q]) | ((uint32_t)f2bf(v[2 * q + 1]) << 16);
    bf16_t* cp = reinterpret_cast<bf16_t*>(Cv) + off;
    if constexpr (W == 8) *reinterpret_cast<uint4*>(cp) = make_uint4(w[0], w[1], w[2], w[3]);
    else *reinterpret_cast<uint2*>(cp) = make_uint2(w[0], w[1]);
  } else {
    float* cp = reinterpret_cast<float*>(Cv) + off;
    float o[W];
    if (OUT == 1 && beta != 0.f) {
      ldw<W>(cp, o);
#pragma unroll
      for (int e = 0; e < W; ++e) o[e] = v[e] + beta * o[e];
    } else {
#pragma unroll
      for (int e = 0; e < W; ++e) o[e] = v[e];
    }
#pragma unroll
    for (int q = 0; q < W / 4; ++q)
      *reinterpret_cast<float4*>(cp + 4 * q) = make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  }
}


// One output tile of one batch entry / K-split ("work item").
struct Work {
  int bz, ks, m0, n0, kbeg, kend, nk;
};
__device__ __forceinline__ Work decode_work(int w, int tiles_n, int tiles, int split_k, int K,
                                            int k_chunk, int bk) {
  Work r;
  const int z = w / tiles, t = w - z * tiles;
  r.bz = z / split_k;
  r.ks = z - r.bz * split_k;
  const int tm = t / tiles_n;
  r.m0 = tm * BM;
  r.n0 = (t - tm * tiles_n) * BN;
  r.kbeg = r.ks * k_chunk;
  r.kend = min(K, r.kbeg + k_chunk);
  r.nk = max(0, (r.kend - r.kbeg + bk - 1) / bk);
  return r;
}

// OUT: 0 bf16, 1 fp32 (C = epi + beta*C), 2 fp32 split-K slab.
// One work item per workgroup; workgroups are remapped so each XCD runs a contiguous range of
// items (tiles sharing an A row-panel share that XCD's L2).
// PIPE 0: double-buffered LDS, operands prefetched one K-step ahead through registers (one
//         barrier per K-step, 2 workgroups/CU) — long K loops.
// PIPE 1: a single LDS stage (write-after-barrier, two barriers per K-step) — short K loops
//         (measured better up to ~24 K-steps); BKT 64: 36 KB, 3 workgroups/CU; BKT 128: 70 KB,
//         2 workgroups/CU, half the latency-bound K-step round trips. A persistent variant
//         (next tile's loads issued before the epilogue) measured slower.
// Epilogue (OUT 0/1): the transposed accumulator runs go to an LDS row-major fp32 tile (16-B
// writes), then 16 threads per row apply the epilogue on 8 columns each (256-B coalesced row
// segments for C / gate / residual). Split-K slabs (OUT 2) are stored straight from registers.
template <bool TA, bool TB, int OUT, int PIPE, int BK>
__global__ __launch_bounds__(NTHREADS, (PIPE == 1 && BK == 64) ? 3 : 2) void gemm_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A0, int64_t lda, int64_t sA,
    const bf16_t* __restrict__ B0, int64_t ldb, int64_t sB, void* __restrict__ Cv, int64_t ldc,
    int64_t sC, int split_k, int k_chunk, int tiles_n, int n_work, Epi epi) {
  constexpr bool DB = PIPE == 0;
  constexpr int TILE_ELEMS = Geom<BK>::TILE;
  constexpr int KCS = Geom<BK>::KCS;
  constexpr int SMEM_ELEMS = (DB ? 4 : 2) * TILE_ELEMS;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM_ELEMS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1, hl = lane >> 5;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  constexpr bool A_KC = !TA;  // A [M][K]
  constexpr bool B_KC = TB;   // B [N][K]
  uint32_t key = 0;
  if (OUT != 2 && epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);

  floatx16 acc[2][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;
  };
  auto mma_tile = [&](const bf16_t* As, const bf16_t* Bs) {
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
        af[a] = load_frag<A_KC, KCS, MC_STRIDE>(As, wm * 64 + a * 32, ks, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b)
        bfr[b] = load_frag<B_KC, KCS, MC_STRIDE>(Bs, wn * 64 + b * 32, ks, lane);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)  // operands swapped: the accumulator holds C^T
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
    }
  };
  uint4 ra[Geom<BK>::Q], rb[Geom<BK>::Q];
  auto load_step = [&](const Work& w, int kt) {
    const int k0 = w.kbeg + kt * BK;
    load_tile<A_KC, BK, 128, NTHREADS>(A0 + w.bz * sA, lda, M, w.kend, w.m0, k0, ra);
    load_tile<B_KC, BK, 128, NTHREADS>(B0 + w.bz * sB, ldb, N, w.kend, w.n0, k0, rb);
  };
  auto store_step = [&](const Work& w, int kt, bf16_t* S) {
    const int k0 = w.kbeg + kt * BK;
    store_tile<A_KC, BK, 128, NTHREADS>(S, ra, M, w.kend, w.m0, k0);
    store_tile<B_KC, BK, 128, NTHREADS>(S + TILE_ELEMS, rb, N, w.kend, w.n0, k0);
  };

  // lane (m = lane & 31, h) of accumulator block (a, b) holds row m, columns 8g + 4h + {0..3}
  auto epilogue = [&](const Work& w) {
    if (OUT == 2) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int gr = w.m0 + wm * 64 + a * 32 + (lane & 31);
        if (gr >= M) continue;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int gc = w.n0 + wn * 64 + b * 32 + 8 * g + 4 * hl;
            if (gc >= N) continue;  // N % 8 == 0: a 4-column run is entirely in or out
            float v[4] = {acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2],
                          acc[a][b][4 * g + 3]};
            store_w<2, 4>(Cv, w.ks * sC + (int64_t)gr * ldc + gc, 0.f, v);
          }
      }
      return;
    }
    constexpr int CTS = BN + 4;         // staging row stride (floats): conflict-free 16-B writes
    constexpr int HALVES = BM * CTS * 4 <= SMEM_ELEMS * 2 ? 1 : 2;  // whole tile or 64-row halves
    constexpr int ROWS = BM / HALVES;
    static_assert(ROWS * CTS * 4 <= SMEM_ELEMS * 2, "staging tile exceeds the LDS");
    float* Ct = reinterpret_cast<float*>(smem);
    const int c8 = (threadIdx.x & 15) * 8;
    const int gc = w.n0 + c8;
#pragma unroll 1
    for (int hf = 0; hf < HALVES; ++hf) {
      __syncthreads();  // operand tile (hf 0) / the previous half (hf 1) consumed
      if (HALVES == 1 || wm == hf) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int r = (HALVES == 1 ? wm * 64 : 0) + a * 32 + (lane & 31);
              *reinterpret_cast<float4*>(Ct + r * CTS + wn * 64 + b * 32 + 8 * g + 4 * hl) =
                  make_float4(acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2],
                              acc[a][b][4 * g + 3]);
            }
      }
      __syncthreads();
      if (gc >= N) continue;
#pragma unroll 2
      for (int r = threadIdx.x >> 4; r < ROWS; r += NTHREADS / 16) {
        const int gr = w.m0 + hf * ROWS + r;
        if (gr >= M) break;
        float v[8];
        ldw<8>(Ct + r * CTS + c8, v);
        epilogue_w<8>(epi, key, N, gr, gc, v);
        store_w<OUT, 8>(Cv, w.bz * sC + (int64_t)gr * ldc + gc, epi.beta, v);
      }
    }
  };

  zero_acc();
  if (DB) {
    const Work w = decode_work(xcd_remap(blockIdx.x, gridDim.x), tiles_n, tiles, split_k, K, k_chunk, BK);
    if (w.nk > 0) {
      load_step(w, 0);
      store_step(w, 0, smem);
    }
    __syncthreads();
    for (int kt = 0; kt < w.nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < w.nk;
      if (more) load_step(w, kt + 1);
      mma_tile(smem + cur * 2 * TILE_ELEMS, smem + cur * 2 * TILE_ELEMS + TILE_ELEMS);
      if (more) store_step(w, kt + 1, smem + (cur ^ 1) * 2 * TILE_ELEMS);
      __syncthreads();
    }
    epilogue(w);
  } else {
    GEMM_TRACE(0);
    const Work w = decode_work(xcd_remap(blockIdx.x, gridDim.x), tiles_n, tiles, split_k, K, k_chunk, BK);
    if (w.nk > 0) load_step(w, 0);
    for (int kt = 0; kt < w.nk; ++kt) {
      if (kt > 0) __syncthreads();  // every wave is done reading the previous K-step
      store_step(w, kt, smem);
      if (kt == 0) GEMM_TRACE(1);
      __syncthreads();
      if (kt + 1 < w.nk) load_step(w, kt + 1);  // in flight during this K-step's MFMAs
      mma_tile(smem, smem + TILE_ELEMS);
    }
    GEMM_TRACE(2);
    epilogue(w);
    GEMM_TRACE(3);
  }
}

// ---------------------------------------------------------------------------------------------
// NT (both operands K-contiguous: the forward Dense layers) with direct global->LDS loads
// (global_load_lds_dwordx4): no VGPR staging and no ds_write pass — the LDS store path is what
// bounds the register-staged kernels (a 128x128x64 step stores 32 KB through ds_write_b128 at
// ~13 cycles/KB, more than the LDS reads and near the MFMA time). Tiles [128][64] bf16 with
// 128-B rows, no padding; 16-B chunk c of row r sits at chunk c ^ ((r >> 1) & 7) (the swizzle is
// applied to each lane's SOURCE address, the DMA destination stays lane-linear, and the fragment
// reads apply the same XOR: conflict-free ds_read_b128). Two stages (64 KB, 2 workgroups/CU);
// the next stage's DMA stays in flight across the barrier (counted vmcnt, raw s_barrier).
// A partial last K-step is zero-filled in LDS after its DMA lands.
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

template <int OUT>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_glds_nt_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A0, int64_t lda, int64_t sA,
    const bf16_t* __restrict__ B0, int64_t ldb, int64_t sB, void* __restrict__ Cv, int64_t ldc,
    int64_t sC, int split_k, int k_chunk, int tiles_n, int n_work, Epi epi) {
  constexpr int BKG = 64;
  constexpr int OPE = 128 * BKG;       // elements per operand tile
  constexpr int STAGE = 2 * OPE;       // A | B
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1, hl = lane >> 5;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const Work w = decode_work(xcd_remap(blockIdx.x, gridDim.x), tiles_n, tiles, split_k, K, k_chunk, BKG);
  const bf16_t* A = A0 + w.bz * sA;
  const bf16_t* B = B0 + w.bz * sB;
  uint32_t key = 0;
  if (OUT != 2 && epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);

  // DMA of K-step kt into stage st: instruction i of this wave fills rows 8(4 wave + i) .. +7
  auto issue = [&](int kt, int st) {
    const int k0 = w.kbeg + kt * BKG;
    bf16_t* SA = smem + st * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = wave * 4 + i;
      const int row = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ swz(row);
      const int kk = min(k0 + c * 8, w.kend - 8);
      const bf16_t* ga = A + (int64_t)min(w.m0 + row, M - 1) * lda + kk;
      const bf16_t* gb = B + (int64_t)min(w.n0 + row, N - 1) * ldb + kk;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ga,
                                       (__attribute__((address_space(3))) void*)(SA + j * 512),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gb,
                                       (__attribute__((address_space(3))) void*)(SA + OPE + j * 512),
                                       16, 0, 0);
    }
  };
  // zero the chunks of a partial K-step that lie past kend (after its DMA landed)
  auto zero_tail = [&](int kt, int st) {
    const int k0 = w.kbeg + kt * BKG;
    bf16_t* SA = smem + st * STAGE;
    for (int e = threadIdx.x; e < 2 * 128 * 8; e += NTHREADS) {
      const int op = e >> 10, row = (e >> 3) & 127, c = e & 7;
      if (k0 + c * 8 >= w.kend)
        *reinterpret_cast<uint4*>(SA + op * OPE + row * BKG + ((c ^ swz(row)) * 8)) =
            make_uint4(0, 0, 0, 0);
    }
  };
  auto frag = [&](const bf16_t* S, int rbase, int ks) {
    const int r = rbase + (lane & 31);
    const int c = (ks * 2 + hl) ^ swz(r);
    return *reinterpret_cast<const bf16x8*>(S + r * BKG + c * 8);
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;

  if (w.nk > 0) issue(0, 0);
  for (int kt = 0; kt < w.nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < w.nk) {
      issue(kt + 1, st ^ 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this K-step's 8 DMAs landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (w.kbeg + (kt + 1) * BKG > w.kend) {
        asm volatile("s_barrier" ::: "memory");
        zero_tail(kt, st);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    asm volatile("s_barrier" ::: "memory");
    const bf16_t* As = smem + st * STAGE;
    const bf16_t* Bs = As + OPE;
    // fragments one k-slice ahead (slice ks + 1's reads in flight under slice ks's MFMAs)
    bf16x8 af[2][2], bfr[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a) af[0][a] = frag(As, wm * 64 + a * 32, 0);
#pragma unroll
    for (int b = 0; b < 2; ++b) bfr[0][b] = frag(Bs, wn * 64 + b * 32, 0);
#pragma unroll
    for (int ks = 0; ks < BKG / 16; ++ks) {
      const int cu = ks & 1;
      if (ks + 1 < BKG / 16) {
#pragma unroll
        for (int a = 0; a < 2; ++a) af[cu ^ 1][a] = frag(As, wm * 64 + a * 32, ks + 1);
#pragma unroll
        for (int b = 0; b < 2; ++b) bfr[cu ^ 1][b] = frag(Bs, wn * 64 + b * 32, ks + 1);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[cu][b], af[cu][a], acc[a][b], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // stage st free again
  }

  // ---------------- epilogue: 64-row halves through the (now idle) LDS
  if (OUT == 2) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int gr = w.m0 + wm * 64 + a * 32 + (lane & 31);
      if (gr >= M) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int gc = w.n0 + wn * 64 + b * 32 + 8 * g + 4 * hl;
          if (gc >= N) continue;
          float v[4] = {acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2],
                        acc[a][b][4 * g + 3]};
          store_w<2, 4>(Cv, w.ks * sC + (int64_t)gr * ldc + gc, 0.f, v);
        }
    }
    return;
  }
  constexpr int CTS = BN + 4;
  static_assert(64 * CTS * 4 <= 2 * STAGE * 2, "staging half exceeds the LDS");
  float* Ct = reinterpret_cast<float*>(smem);
  const int c8 = (threadIdx.x & 15) * 8;
  const int gc = w.n0 + c8;
  // Every global operand of the epilogue (bias, gate, residual, the old C of C += ...) is loaded
  // before the first store of its half: one in-order vmcnt retires loads and stores together, so
  // a load issued behind stores waits for all of them. alpha, bias, relu, gate and the residual
  // are applied here, dropout through epilogue_w with the rest of epi: epilogue_w's order.
  constexpr int RPT = 64 / (NTHREADS / 16);  // rows per thread per half
  const int gcl = min(gc, N - 8);            // clamped: unpredicated loads keep vmcnt exact
  float bias_r[8];
  if (epi.bias) ldw<8>(epi.bias + gcl, bias_r);
  Epi rest = epi;
  rest.alpha = 1.f;
  rest.bias = nullptr;
  rest.act = MMT_ACT_NONE;
  rest.gate = nullptr;
  rest.residual = nullptr;
  const bool old_c = OUT == 1 && epi.beta != 0.f;
#pragma unroll 1
  for (int hf = 0; hf < 2; ++hf) {
    float res_r[RPT][8], c_r[RPT][8];
    uint4 gate_r[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int gr = min(w.m0 + hf * 64 + (threadIdx.x >> 4) + i * (NTHREADS / 16), M - 1);
      if (epi.residual) {
        const int64_t ro = (int64_t)gr * epi.ld_res + gcl;
        if (epi.res_f32) ldw<8>(reinterpret_cast<const float*>(epi.residual) + ro, res_r[i]);
        else ldw<8>(reinterpret_cast<const bf16_t*>(epi.residual) + ro, res_r[i]);
      }
      if (epi.gate)
        gate_r[i] = *reinterpret_cast<const uint4*>(epi.gate + (int64_t)gr * epi.ld_gate + gcl);
      if (old_c) ldw<8>(reinterpret_cast<const float*>(Cv) + w.bz * sC + (int64_t)gr * ldc + gcl, c_r[i]);
    }
    __syncthreads();
    if (wm == hf) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(Ct + (a * 32 + (lane & 31)) * CTS + wn * 64 + b * 32 +
                                       8 * g + 4 * hl) =
                make_float4(acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2],
                            acc[a][b][4 * g + 3]);
    }
    __syncthreads();
    if (gc >= N) continue;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = (threadIdx.x >> 4) + i * (NTHREADS / 16);
      const int gr = w.m0 + hf * 64 + r;
      if (gr >= M) break;
      float v[8];
      ldw<8>(Ct + r * CTS + c8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= epi.alpha;
      if (epi.bias)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bias_r[e];
      if (epi.act == MMT_ACT_RELU)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      if (epi.gate) {
        const uint32_t gw[4] = {gate_r[i].x, gate_r[i].y, gate_r[i].z, gate_r[i].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float g0 = __uint_as_float(gw[q] << 16), g1 = __uint_as_float(gw[q] & 0xffff0000u);
          v[2 * q] *= (g0 > 0.f) ? epi.gate_scale : 0.f;
          v[2 * q + 1] *= (g1 > 0.f) ? epi.gate_scale : 0.f;
        }
      }
      epilogue_w<8>(rest, key, N, gr, gc, v);
      if (epi.residual)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += res_r[i][e];
      if (old_c)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += epi.beta * c_r[i][e];
      store_w<OUT, 8>(Cv, w.bz * sC + (int64_t)gr * ldc + gc, 0.f, v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Large-tile variant for big launches: 256 x 192 output tile, 8 waves (4 along M x 2 along N,
// 64 x 96 each = 2 x 3 MFMA blocks), K-step 64, double-buffered LDS (2 x 64.5 KB) with operands
// prefetched one K-step ahead through registers, one workgroup per CU. Against the 128 x 128
// tile it moves 1/110 instead of 1/64 operand bytes per flop through the per-CU load
// path, which bounds the small tile (tools/gemm_trace.cpp: per-K-step time grows with the bytes
// per step, not with occupancy). 192 divides every N of the path (384, 768, 1152, 1536, 2304,
// 3072), so the last N tile is never partial there.
constexpr int BM2 = 256, BN2 = 192, BK2 = 64, NT2 = 512;

template <bool TA, bool TB, int OUT>
__global__ __launch_bounds__(NT2, 1) void gemm_big_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A0, int64_t lda, int64_t sA,
    const bf16_t* __restrict__ B0, int64_t ldb, int64_t sB, void* __restrict__ Cv, int64_t ldc,
    int64_t sC, int split_k, int k_chunk, int tiles_n, int n_work, Epi epi) {
  constexpr bool A_KC = !TA, B_KC = TB;
  constexpr int A_MCS = BM2 + 8, B_MCS = BN2 + 8, KCS = BK2 + 8;
  constexpr int TA_E = A_KC ? BM2 * KCS : BK2 * A_MCS;
  constexpr int TB_E = B_KC ? BN2 * KCS : BK2 * B_MCS;
  constexpr int STAGE = TA_E + TB_E;
  constexpr int QA = BM2 * BK2 / 8 / NT2, QB = BN2 * BK2 / 8 / NT2;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1, hl = lane >> 5;
  const int tiles = ((M + BM2 - 1) / BM2) * tiles_n;
  uint32_t key = 0;
  if (OUT != 2 && epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);

  // work item
  const int wi = xcd_remap(blockIdx.x, gridDim.x);
  const int z = wi / tiles, t = wi - z * tiles;
  const int bz = z / split_k, ks_id = z - bz * split_k;
  const int tm = t / tiles_n;
  const int m0 = tm * BM2, n0 = (t - tm * tiles_n) * BN2;
  const int kbeg = ks_id * k_chunk, kend = min(K, kbeg + k_chunk);
  const int nk = max(0, (kend - kbeg + BK2 - 1) / BK2);
  const bf16_t* A = A0 + bz * sA;
  const bf16_t* B = B0 + bz * sB;

  floatx16 acc[2][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;

  uint4 ra[QA], rb[QB];
  auto load_step = [&](int kt) {
    const int k0 = kbeg + kt * BK2;
    load_tile<A_KC, BK2, BM2, NT2>(A, lda, M, kend, m0, k0, ra);
    load_tile<B_KC, BK2, BN2, NT2>(B, ldb, N, kend, n0, k0, rb);
  };
  auto store_step = [&](int kt, bf16_t* S) {
    const int k0 = kbeg + kt * BK2;
    store_tile<A_KC, BK2, BM2, NT2>(S, ra, M, kend, m0, k0);
    store_tile<B_KC, BK2, BN2, NT2>(S + TA_E, rb, N, kend, n0, k0);
  };
  auto mma_tile = [&](const bf16_t* As, const bf16_t* Bs) {
#pragma unroll
    for (int ks = 0; ks < BK2 / 16; ++ks) {
      bf16x8 af[2], bfr[3];
#pragma unroll
      for (int a = 0; a < 2; ++a)
        af[a] = load_frag<A_KC, KCS, A_MCS>(As, wm * 64 + a * 32, ks, lane);
#pragma unroll
      for (int b = 0; b < 3; ++b)
        bfr[b] = load_frag<B_KC, KCS, B_MCS>(Bs, wn * 96 + b * 32, ks, lane);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b)  // operands swapped: the accumulator holds C^T
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
    }
  };

  if (nk > 0) {
    load_step(0);
    store_step(0, smem);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_step(kt + 1);
    mma_tile(smem + cur * STAGE, smem + cur * STAGE + TA_E);
    if (more) store_step(kt + 1, smem + (cur ^ 1) * STAGE);
    __syncthreads();
  }

  // ---------------- epilogue (lane (m = lane & 31, h) of block (a, b): row m, columns 8g+4h+{0..3})
  if (OUT == 2) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int gr = m0 + wm * 64 + a * 32 + (lane & 31);
      if (gr >= M) continue;
#pragma unroll
      for (int b = 0; b < 3; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int gc = n0 + wn * 96 + b * 32 + 8 * g + 4 * hl;
          if (gc >= N) continue;
          float v[4] = {acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2],
                        acc[a][b][4 * g + 3]};
          store_w<2, 4>(Cv, ks_id * sC + (int64_t)gr * ldc + gc, 0.f, v);
        }
    }
    return;
  }
  // 64-row chunks through an LDS fp32 tile [64][196]; chunk c comes from the two waves wm == c
  constexpr int CTS = BN2 + 4;
  static_assert(64 * CTS * 4 <= 2 * STAGE * 2, "staging chunk exceeds the LDS");
  float* Ct = reinterpret_cast<float*>(smem);
  constexpr int GPR = BN2 / 8;  // 8-column groups per row
#pragma unroll 1
  for (int c = 0; c < BM2 / 64; ++c) {
    if (c > 0) __syncthreads();  // previous chunk consumed
    if (wm == c) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<float4*>(Ct + (a * 32 + (lane & 31)) * CTS + wn * 96 + b * 32 +
                                       8 * g + 4 * hl) =
                make_float4(acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2],
                            acc[a][b][4 * g + 3]);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * GPR; e += NT2) {
      const int r = e / GPR, g8 = (e - r * GPR) * 8;
      const int gr = m0 + c * 64 + r, gc = n0 + g8;
      if (gr >= M || gc >= N) continue;
      float v[8];
      ldw<8>(Ct + r * CTS + g8, v);
      epilogue_w<8>(epi, key, N, gr, gc, v);
      store_w<OUT, 8>(Cv, bz * sC + (int64_t)gr * ldc + gc, epi.beta, v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent 256 x BN NT kernel (forward Dense layers and, with the transposed weight shadow, the
// input gradients): one 512-thread workgroup per CU walks a strided list of output tiles; the
// (tile, K-step) sequence is flattened so the first K-step of the NEXT tile is DMA'd while the
// current tile finishes its last K-step and runs its epilogue (no per-tile prologue bubble, the
// epilogue's store tail overlaps the next tile's loads).
//  * 8 waves as 4 (M) x 2 (N); wave tile 64 x W (W = BN/2), v_mfma_f32_16x16x32_bf16 with the
//    operands swapped (accumulator = C^T: lane holds 4 consecutive columns of one row).
//  * B fragment rows are permuted so that lane group q = lane>>4 owns the W/4 CONTIGUOUS columns
//    q*W/4 .. q*W/4+W/4-1 of its row across the W/16 fragments: the epilogue stores 16-B vectors
//    straight from registers (no LDS round trip, which the next tile's DMA is using).
//  * operands DMA'd global->LDS (global_load_lds_dwordx4) into unpadded [rows][64] bf16 images
//    (128-B rows); the 16-B chunk c of row r sits at c ^ f(r), applied to each lane's SOURCE
//    address (the DMA destination is lane-linear) and to the fragment reads. f_A(r) = r & 6 and
//    f_B(r) = (r & 2) | bit(r, log2(W/4)) << 2 make every ds_read_b128 of both the plain A rows
//    and the permuted B rows conflict-free (exhaustive check over the 16-lane groups).
//  * two LDS stages; one K-step's DMA is in flight during the previous K-step's MFMAs, waited
//    for by a counted vmcnt (the previous tile's epilogue stores, issued after it, are counted
//    in the immediate) and a raw s_barrier, never vmcnt(0) in the loop.
// Requires K % 64 == 0 and N % BN == 0 (checked by mmt_gemm); rows past M are clamped on load
// and not stored.
constexpr int NT3 = 512;
constexpr int NT_BIAS_LDS = 3072;  // floats of bias held in LDS (every step shape: N <= 3072)
#ifndef NT_SH256  // stashed output chunks of the bf16 256-wide tile (0: all stored by the epilogue;
#define NT_SH256 0  // measured: 4 and 8 slower at M = 70656, K = 384 and 1536)
#endif

// buffer_load_dwordx4 ... lds of 16 B per lane: byte voffset + soffset inside [base, base + bytes)
// (out-of-range lanes read zeros) into the wave-uniform LDS address lds (+ 16 * lane).
__device__ __forceinline__ void dma16(const void* base, int64_t bytes, void* lds, int voffset,
                                      int soffset) {
#if defined(__HIP_DEVICE_COMPILE__)  // the buffer-resource type exists only in the device pass
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(base), (short)0, (int)min(bytes, (int64_t)0x7ffffff0), 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           voffset, soffset, 0, 0);
#endif
}

template <int BN, int OUT, int SHV, int NS, bool CS = false, bool GBITS = false, bool KB = false>
__global__ __launch_bounds__(NT3, 1) void gemm_nt256_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
    int64_t ldb, void* __restrict__ Cv, int64_t ldc, int tiles_n, int n_tiles, int xcd_order,
    Epi epi) {
  constexpr int W = BN / 2, NF = W / 16, Q = W / 4;
  static_assert(NF % 2 == 0, "column fragments come in pairs");
  constexpr int A_BYTES = 256 * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int GA = 4, GB = BN / 64, G = GA + GB;  // DMA instructions per wave per K-step
  // 16-B output chunks per lane per tile (CPM per 16-row fragment). The last SH of them (SHV; -1:
  // all) are held in registers (the stash) and stored SPS per K-step during the next tile
  // (NSTEPS K-steps); the first EI are stored by the epilogue itself.
  constexpr int CPM = OUT == 0 ? Q / 8 : Q / 4, E = 4 * CPM;
  constexpr int SH = SHV < 0 ? E : SHV, EI = E - SH;
  constexpr bool STASH = SH > 0;
  constexpr int SPS = 4, NSTEPS = SH / SPS;
  static_assert(SH % SPS == 0 && SH <= E && EI % 2 == 0, "stash chunks");
  static_assert(NS == 2 || (NS == 3 && STASH && EI == 0), "3 stages only with the full stash");
  static_assert(!CS || OUT == 0, "column sums of bf16 outputs only");
  // ONE LDS object: the operand stages, then the bias vector (the host sends N > NT_BIAS_LDS with
  // a bias elsewhere; staged once per launch — an epilogue global load issued behind the previous
  // chunks' stores waits for all of them on the one in-order vmcnt), then the CS column sums.
  // Separate __shared__ arrays make the compiler put a vmcnt(0) in front of every ds_read that
  // follows a buffer_load ... lds (it cannot tell the objects apart), serialising the K-loop.
  constexpr int CS_FLOATS = CS ? 4 * BN : 0;
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE + 4 * (NT_BIAS_LDS + CS_FLOATS)];
  float* const s_bias = reinterpret_cast<float*>(smem + NS * STAGE);
  float (*const s_cs)[BN] = reinterpret_cast<float (*)[BN]>(s_bias + NT_BIAS_LDS);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nk = K / 64;
  // Tile order. xcd_order: each XCD owns one contiguous eighth of the (row-panel major) tile
  // range for the whole launch, its workgroups (dispatch is round-robin over the 8 XCDs, so
  // blockIdx & 7 is the XCD) striding through it together: an A row panel is fetched into ONE
  // XCD's L2 and consumed there by its tn column tiles. Otherwise: strided over the whole grid
  // with the bijective remap (a panel can straddle two XCDs at every stride step).
  int first, stride, limit = n_tiles;
  if (xcd_order && (gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7, per = gridDim.x >> 3;
    first = (int)((int64_t)n_tiles * xcd / 8) + (blockIdx.x >> 3);
    limit = (int)((int64_t)n_tiles * (xcd + 1) / 8);
    stride = per;
  } else {
    first = xcd_remap(blockIdx.x, gridDim.x);
    stride = gridDim.x;
  }
  const int n_mine = first < limit ? (limit - first + stride - 1) / stride : 0;
  const int S = n_mine * nk;
  uint32_t key = 0;
  if (epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);
  // The epilogue applies alpha, bias (from LDS), relu and the gate (its loads issued one fragment
  // row ahead, before the previous row's stores) itself; dropout and residual go through
  // epilogue_w with the rest of epi. Same arithmetic, same order as epilogue_w.
  Epi rest = epi;
  rest.alpha = 1.f;
  rest.bias = nullptr;
  rest.act = MMT_ACT_NONE;
  rest.gate = nullptr;
  rest.relu_bits = nullptr;
  rest.gate_bits = nullptr;
  constexpr bool BITS = BN == 256;  // the 1-bit gate layout is this tile's lane layout (Q = 32)
  static_assert(!GBITS || BITS, "1-bit gate only on 256-wide tiles");
  constexpr bool RBITS = BITS && !CS && !GBITS;  // relu_bits writer (a forward launch)
  // KB (keep_bits launches, a separate instantiation: the runtime-checked form cost the default
  // MLP-up kernel 3 % through scalar-register spills): the dropout keeps precomputed in the
  // relu_bits layout (mmt_gemm_dropout_keep_bits) replace the epilogue's counter-hash draws; the
  // tile's word is loaded at its first K-step and held until its epilogue
  static_assert(!KB || (RBITS && OUT == 0), "keep_bits only in the bf16 relu_bits launch");
  constexpr bool KBITS = KB;
  if (KBITS) rest.rng = nullptr;
  uint4 kbw = make_uint4(0u, 0u, 0u, 0u);
  // GBITS: the gate comes as bits (gate_bits); otherwise as bf16 rows (gate) — one of the two
  // compiled per instantiation (both at once spill registers in the column-sum variant)

  auto fA = [](int r) { return r & 6; };
  auto fB = [](int r) { return (r & 2) | (((r >> 3) & 1) << 2); };
  // one DMA piece (1 KB per wave) of K-step position (m0, n0, k0) into stage st:
  // pieces 0..GA-1 are A rows 8j..8j+7 (j = wave*GA + p), the rest B rows. buffer_load ... lds
  // with the tile's panel as the buffer: the per-lane byte offsets (row, swizzled chunk) are
  // fixed for the kernel, the panel base and k0 are scalars, so a piece costs no VALU; A rows
  // past M fall outside the buffer's range and read as zeros.
  int voff[G];
#pragma unroll
  for (int p = 0; p < G; ++p) {
    const int j = p < GA ? wave * GA + p : wave * GB + (p - GA);
    const int row = 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ (p < GA ? fA(row) : fB(row));
    voff[p] = row * (int)((p < GA ? lda : ldb) * 2) + c * 16;
  }
  auto piece = [&](int m0, int n0, int k0, int st, int p) {
    char* S0 = smem + st * STAGE;
    if (p < GA)
      dma16(A + (int64_t)m0 * lda, (int64_t)(M - m0) * lda * 2, S0 + (wave * GA + p) * 1024,
            voff[p], k0 * 2);
    else
      dma16(B + (int64_t)n0 * ldb, (int64_t)BN * ldb * 2,
            S0 + A_BYTES + (wave * GB + (p - GA)) * 1024, voff[p], k0 * 2);
  };
  auto position = [&](int s, int& m0, int& n0, int& k0) {
    const int i = s / nk, kt = s - i * nk;
    const int tile = first + i * stride;
    const int tm = tile / tiles_n;
    m0 = tm * 256;
    n0 = (tile - tm * tiles_n) * BN;
    k0 = kt * 64;
  };

  typedef float floatx4 __attribute__((ext_vector_type(4)));
  floatx4 acc[4][NF];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NF; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment row offsets (bytes) and swizzles, fixed for the kernel
  const int l15 = lane & 15, lq = lane >> 4;
  int a_off[4], a_sw[4], b_off[NF], b_sw[NF];
#pragma unroll
  for (int mf = 0; mf < 4; ++mf) {
    const int r = wm * 64 + mf * 16 + l15;
    a_off[mf] = r * 128;
    a_sw[mf] = fA(r);
  }
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int r = wn * W + 32 * (nf >> 1) + 8 * (l15 >> 2) + 4 * (nf & 1) + (l15 & 3);
    b_off[nf] = A_BYTES + r * 128;
    b_sw[nf] = fB(r);
  }

  // Output stash (STASH): the finished tile's epilogue values, bf16-packed (OUT 0) or fp32, as
  // 16-B chunks ci = mf * CPM + c; chunk ci covers row srow + 16 mf, columns sgc + 32c (bf16) /
  // sgc + 32(c >> 1) + 4(c & 1) (fp32): the four lq lanes of a row store 64 contiguous bytes
  // (bf16) or 128 (fp32) per instruction.
  uint32_t stash[STASH ? SH : 1][4];
  int sk = NSTEPS;            // next K-step's store group (NSTEPS: nothing left to store)
  int srow = 0, sgc = 0;      // this lane's first row / first column of the stashed tile
  auto stash_store = [&](int ci) {  // stash entry ci = output chunk EI + ci
    const int mf = (EI + ci) / CPM, c = EI + ci - mf * CPM;
    const int gr = srow + 16 * mf;
    if (gr < M) {
      const int64_t off = (int64_t)gr * ldc + sgc + (OUT == 0 ? 32 * c : 32 * (c >> 1) + 4 * (c & 1));
      const uint4 u = make_uint4(stash[ci][0], stash[ci][1], stash[ci][2], stash[ci][3]);
      // plain stores: non-temporal ones measured twice this kernel's time
      if (OUT == 0) *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(Cv) + off) = u;
      else *reinterpret_cast<uint4*>(reinterpret_cast<float*>(Cv) + off) = u;
    }
  };

  // Waves 0-3 issue the next K-step's DMA in the first half of the MFMAs and waves 4-7 (their
  // SIMD partners) in the second, so one wave of each SIMD pair always has MFMAs to issue while
  // the other stalls on DMA issue; the stash stores go in the other half.
  const int hl = 0;
  // MFMAs of the K-step in stage st. The next K-step's G DMA pieces (into the other stage, free
  // since the barrier that opened this K-step) are issued two per M-fragment block in the first
  // half: a piece costs its wave ~100 issue cycles, which the SIMD's partner wave fills with
  // MFMAs instead of both waves stalling on a burst of issues at the top of the K-step.
  auto compute = [&](int st, bool nxt, int nst, int nm0, int nn0, int nk0) {
    const char* S0 = smem + st * STAGE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 4 * h + lq;
      bf16x8 af[4], bfr[NF];
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
        af[mf] = *reinterpret_cast<const bf16x8*>(S0 + a_off[mf] + ((c ^ a_sw[mf]) << 4));
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
        bfr[nf] = *reinterpret_cast<const bf16x8*>(S0 + b_off[nf] + ((c ^ b_sw[nf]) << 4));
#pragma unroll
      for (int mf = 0; mf < 4; ++mf) {
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nf], af[mf], acc[mf][nf], 0, 0, 0);
        if (h == hl && nxt) {
          if (2 * mf < G) piece(nm0, nn0, nk0, nst, 2 * mf);
          if (2 * mf + 1 < G) piece(nm0, nn0, nk0, nst, 2 * mf + 1);
        }
        if (STASH && h != hl && sk < NSTEPS) {
#pragma unroll
          for (int j = 0; j < NSTEPS; ++j)
            if (sk == j) stash_store(j * SPS + mf);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // lane (row l15 of fragment mf, group lq) holds columns 32 (nf >> 1) + 8 lq + 4 (nf & 1) + r of
  // the wave's W: runs of 8 columns, the four lq lanes' runs adjacent (B-fragment row order
  // above), so each store instruction writes 64 contiguous bytes per row instead of four 16-B
  // pieces at a 64-B stride
  auto epilogue = [&](int tile) {
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int gc0 = tn * BN + wn * W + 8 * lq;
    float cs[CS ? Q : 1];  // CS: this lane's column sums over its rows of the tile
    if constexpr (CS)
#pragma unroll
      for (int j = 0; j < Q; ++j) cs[j] = 0.f;
    if (STASH) {  // store what is left of the previous stash (K-loops shorter than NSTEPS)
#pragma unroll
      for (int j = 0; j < NSTEPS; ++j)
        if (j >= sk)
#pragma unroll
          for (int b = 0; b < SPS; ++b) stash_store(j * SPS + b);
      sk = 0;
      srow = tm * 256 + wm * 64 + l15;
      sgc = gc0;
    }
    // gate rows, double-buffered one fragment row ahead (rows clamped into range: an unpredicated
    // load keeps the compiler's vmcnt counting exact)
    uint4 gq[2][Q / 8];
    auto gate_load = [&](int mf, int buf) {
      const int gr = min(tm * 256 + wm * 64 + mf * 16 + l15, M - 1);
#pragma unroll
      for (int c8 = 0; c8 < Q / 8; ++c8)
        gq[buf][c8] = *reinterpret_cast<const uint4*>(epi.gate + (int64_t)gr * epi.ld_gate + gc0 + 32 * c8);
    };
    // 1-bit gate / relu words (include/mmt_api.h layout): this lane's 4 rows (mf) x 32 columns
    // are one uint4 at [(tm * 64 + wm * 16 + l15)][tn * 8 + wn * 4 + lq]: one 16-B load / store
    // per lane per tile, the 4 lq lanes of a row group writing 64 contiguous bytes
    const int64_t bidx = (int64_t)(tm * 64 + wm * 16 + l15) * (N / 32) + (tn * 8 + wn * 4 + lq);
    uint4 gbw = make_uint4(0u, 0u, 0u, 0u);
    if (GBITS && epi.gate_bits) gbw = reinterpret_cast<const uint4*>(epi.gate_bits)[bidx];
    uint32_t rbw[4] = {0u, 0u, 0u, 0u};  // relu_bits words of this lane's 4 rows
    if (!GBITS && epi.gate) gate_load(0, 0);
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      const int gr = tm * 256 + wm * 64 + mf * 16 + l15;
      if (!GBITS && epi.gate && mf < 3) gate_load(mf + 1, (mf + 1) & 1);
      if (gr < M) {
#pragma unroll
        for (int c8 = 0; c8 < Q / 8; ++c8) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = acc[mf][(8 * c8 + e) >> 2][e & 3] * epi.alpha;
          const int gc = gc0 + 32 * c8;
          if (epi.bias) {
            float bb[8];
            const float4 b0 = *reinterpret_cast<const float4*>(s_bias + gc);
            const float4 b1 = *reinterpret_cast<const float4*>(s_bias + gc + 4);
            bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
            bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bb[e];
          }
          if (epi.act == MMT_ACT_RELU)
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          if (!GBITS && epi.gate) {
            const uint4 u = gq[mf & 1][c8];
            const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float g0 = __uint_as_float(w[q] << 16), g1 = __uint_as_float(w[q] & 0xffff0000u);
              v[2 * q] *= (g0 > 0.f) ? epi.gate_scale : 0.f;
              v[2 * q + 1] *= (g1 > 0.f) ? epi.gate_scale : 0.f;
            }
          }
          if (GBITS && epi.gate_bits) {
            const uint32_t w = (mf == 0 ? gbw.x : mf == 1 ? gbw.y : mf == 2 ? gbw.z : gbw.w) >> (8 * c8);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= ((w >> e) & 1u) ? epi.gate_scale : 0.f;
          }
          if (KBITS) {
            const uint32_t w = (mf == 0 ? kbw.x : mf == 1 ? kbw.y : mf == 2 ? kbw.z : kbw.w) >> (8 * c8);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = ((w >> e) & 1u) ? v[e] * epi.drop_scale : 0.f;
          }
          epilogue_w<8>(rest, key, N, gr, gc, v);
          if (RBITS && epi.relu_bits)  // stored bf16 > 0 <=> v > 0 (bf16 keeps fp32's exponent range)
#pragma unroll
            for (int e = 0; e < 8; ++e) rbw[mf] |= (v[e] > 0.f ? 1u : 0u) << (8 * c8 + e);
          if constexpr (CS)  // the values as stored (bf16)
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[8 * c8 + e] += __uint_as_float((uint32_t)f2bf(v[e]) << 16);
          if (STASH && mf * CPM + (OUT == 0 ? c8 : 2 * c8) >= EI) {
            const int ci = mf * CPM + (OUT == 0 ? c8 : 2 * c8) - EI;  // stash entry
            if (OUT == 1 && epi.beta != 0.f) {
              float o[8];
              ldw<8>(reinterpret_cast<const float*>(Cv) + (int64_t)gr * ldc + gc0 + 32 * c8, o);
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] += epi.beta * o[e];
            }
            if (OUT == 0) {
              uint32_t* d = stash[ci];
#pragma unroll
              for (int q = 0; q < 4; ++q)
                d[q] = (uint32_t)f2bf(v[2 * q]) | ((uint32_t)f2bf(v[2 * q + 1]) << 16);
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) stash[ci + (q >> 2)][q & 3] = __float_as_uint(v[q]);
            }
            continue;
          }
          store_w<OUT, 8>(Cv, (int64_t)gr * ldc + gc0 + 32 * c8, epi.beta, v);
        }
      }
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[mf][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if (RBITS && epi.relu_bits)
      reinterpret_cast<uint4*>(epi.relu_bits)[bidx] = make_uint4(rbw[0], rbw[1], rbw[2], rbw[3]);
    if constexpr (CS) {
      // sum over the 16 row lanes (l15) of each DPP row: xor 1, xor 2, half-row and row mirrors
#pragma unroll
      for (int j = 0; j < Q; ++j) {
        float x = cs[j];
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xf, 0xf, false));
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xf, 0xf, false));
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xf, 0xf, false));
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xf, 0xf, false));
        cs[j] = x;
      }
      if (l15 == 0)
#pragma unroll
        for (int j = 0; j < Q; ++j) s_cs[wm][wn * W + 32 * (j >> 3) + 8 * lq + (j & 7)] = cs[j];
      // LDS only (no fence: the epilogue's global stores stay in flight)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (threadIdx.x < BN)
        epi.colsum[(int64_t)tm * N + tn * BN + threadIdx.x] =
            s_cs[0][threadIdx.x] + s_cs[1][threadIdx.x] + s_cs[2][threadIdx.x] + s_cs[3][threadIdx.x];
    }
  };

  if (S == 0) return;
#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (q < S) {
      int m0, n0, k0;
      position(q, m0, n0, k0);
#pragma unroll
      for (int p = 0; p < G; ++p) piece(m0, n0, k0, q, p);
    }
  // published by the loop's first barrier, long before the first epilogue
  if (epi.bias)  // N <= NT_BIAS_LDS (nt_bn)
    for (int i = threadIdx.x; i < N; i += NT3) s_bias[i] = epi.bias[i];
  // vmcnt(n) for the wave-uniform counts the loop can need
  auto wait_vm = [](int n) {
    if (n == SPS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SPS) : "memory");
    else if (n == 2 * SPS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * SPS) : "memory");
    else if (n == G) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    else if (n == G + SPS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G + SPS) : "memory");
    else if (n == G + 2 * SPS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G + 2 * SPS) : "memory");
    else if (n == EI && EI > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EI) : "memory");
    else if (n == EI + SPS && EI > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(EI + SPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  // One barrier per K-step: K-step s's DMA was issued during K-step s-1's MFMAs; the barrier
  // after its vmcnt wait both publishes it and frees the other stage for K-step s+1's DMA.
  // The epilogue of tile i runs at the top of the next tile's first iteration (its stores stay
  // in flight across that K-step: vmcnt(E)).
  bool pend = false, counted = false;  // counted: the last tile was full (exact store counts)
  int sc1 = 0, sc2 = 0;  // exact stash stores (0 or SPS) issued by the last two K-steps
  int ptile = 0;
  for (int s = 0; s < S; ++s) {
    const int st = NS == 2 ? (s & 1) : s % 3;
    const int i = s / nk, kt = s - i * nk;
    NT_STEP(s, 0);
    if (pend) {
      epilogue(ptile);
      NT_TRACE(i - 1, 2);
      pend = false;
      counted = (ptile / tiles_n) * 256 + 256 <= M;
      // younger than K-step s's DMA: the previous K-step's stash stores and this epilogue's EI
      // immediate stores (exact only for a full tile)
      if (STASH) wait_vm(EI > 0 ? (counted ? EI + sc1 : 0)
                                : NS == 2 ? sc1 : (s + 1 < S ? G : 0) + sc1 + sc2);  // see below
      else if (counted) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(E) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (STASH) {
      // younger than K-step s's DMA (issued in K-step s-NS+1's first MFMA half): the stash
      // stores of the later K-steps' second halves and, with 3 stages, K-step s+1's DMA
      wait_vm(NS == 2 ? sc1 : (s + 1 < S ? G : 0) + sc1 + sc2);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    NT_STEP(s, 1);
    asm volatile("s_barrier" ::: "memory");  // K-step s landed for every wave; stage st^1 free
    NT_STEP(s, 2);
    if (KBITS && kt == 0) {  // after the previous tile's epilogue (its word is in kbw until then)
      const int tile = first + i * stride, tm = tile / tiles_n, tn = tile - tm * tiles_n;
      kbw = reinterpret_cast<const uint4*>(epi.keep_bits)[(int64_t)(tm * 64 + wm * 16 + l15) * (N / 32) +
                                                          (tn * 8 + wn * 4 + lq)];
    }
    if (kt == 0) NT_TRACE(i, 0);
    if (s == 0) NT_CLK(0);
    int nm0 = 0, nn0 = 0, nk0 = 0;
    const bool nxt = s + NS - 1 < S;
    if (nxt) position(s + NS - 1, nm0, nn0, nk0);
    compute(st, nxt, NS == 2 ? (st ^ 1) : (st + 2) % 3, nm0, nn0, nk0);
    const bool stored = STASH && sk < NSTEPS;
    if (stored) ++sk;
    sc2 = sc1;
    sc1 = stored && counted ? SPS : 0;  // counted: the stashed tile is full (no skipped rows)
    NT_STEP(s, 3);
    if (kt == nk - 1) {
      NT_TRACE(i, 1);
      pend = true;
      ptile = first + i * stride;
    }
  }
  epilogue(ptile);
  if (STASH)
#pragma unroll
    for (int ci = 0; ci < SH; ++ci) stash_store(ci);
  NT_TRACE(n_mine - 1, 2);
  NT_CLK(1);
}

// ---------------------------------------------------------------------------------------------
// Narrow-output NT kernel (the products hipBLASLt used to run: the MLP and QKV input gradients
// 141,312 x 384 x 1536 / 149,504 x 384 x 1152, the frozen T5's FF output + residual
// 16,384 x 768 x 3072, and the T5 FF input relu(16,384 x 3072 x 768)): C = epi(A . B^T), bf16,
// MT x BN tiles (BN 384 or 192), K-steps of 64.
// The A operand streams from HBM once; B (N x K, 1.2 MB at N = 384) is re-read from L2 by every
// tile. An HBM miss costs ~3 us under full load, so A needs more than one K-step of DMA in flight
// per CU, and with one in-order vmcnt per wave the B loads must never sit behind a younger A
// load that the same barrier does not need. Hence separate LDS rings: NSA A stages (DMA issued
// NSA - 1 K-steps ahead) and two B stages (one ahead), issued per K-step as [B(s+1), A(s+NSA-1)]:
// the barrier of K-step s waits for B(s) with vmcnt(A pieces + stores younger than it), which
// leaves A(s+NSA-2) in flight across the barrier and has retired A(s) long before.
//  * one 512-thread workgroup per CU, persistent over a strided (XCD-contiguous, row-panel-major)
//    tile list: the BN-column tiles of one A row panel run together on one XCD (one HBM fetch);
//    the (tile, K-step) sequence is flattened, so the next tile's loads overlap this tile's end;
//  * 8 waves as (MT/WM) x (BN/96), wave tile WM x 96 of v_mfma_f32_32x32x16_bf16, operands
//    swapped so the accumulator is C^T (lane = output row, 16 columns in runs of 4);
//  * operands DMA'd global->LDS (buffer_load ... lds, 1 KB per wave-instruction, buffer
//    resources rebuilt per tile) into unpadded [rows][64] bf16 images, 16-B chunk c of row r at
//    c ^ ((r >> 1) & 7) (source-address swizzle; conflict-free fragment ds_read_b128: each of the
//    instruction's 16-lane groups takes 16 distinct (row parity, chunk) bank sets. Through round 6
//    it was c ^ (r & 7), which pairs rows r and r + 8 of a group on one bank set: 2-way conflicts
//    on every fragment read, half the kernel's LDS cycles; MLP dX 218 -> 211 us);
//  * the host plans the launch so no round of the persistent grid is mostly idle (mmt_gemm);
//  * epilogue from registers: v_permlane32_swap pairs the two half-waves' column runs into 8
//    contiguous columns per lane (16-B residual loads and C stores).
// Requires N % BN == 0, K % 64 == 0; rows past M read zeros and are not stored.
constexpr int NTW_NT = 512;
template <int MT, int BN, int EP>  // EP: 0 plain, 1 + bf16 residual, 2 relu
__global__ __launch_bounds__(NTW_NT, 2) void gemm_ntw_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
    int64_t ldb, bf16_t* __restrict__ C, int64_t ldc, const bf16_t* __restrict__ R, int64_t ldr,
    int tiles_n, int n_tiles) {
  constexpr int WGN = BN / 96, WGM = 8 / WGN, WM = MT / WGM, MB = WM / 32, NB = 3;
  static_assert(BN % 96 == 0 && 8 % WGN == 0 && WM % 32 == 0, "tile / wave geometry");
  constexpr int A_ST = MT * 128, B_ST = BN * 128;
  constexpr int NSA_FIT = (163840 - 2 * B_ST) / A_ST, NSA = NSA_FIT > 4 ? 4 : NSA_FIT;
  static_assert(NSA >= 2, "LDS");
  constexpr int PA = MT / 64, PB = BN / 64;  // DMA pieces (8 rows x 128 B) per wave per K-step
  static_assert(MT % 64 == 0 && BN % 64 == 0, "pieces");
  constexpr int E = MB * NB * 2;             // 16-B C stores per lane per tile
  static_assert(PA * (NSA - 2 > 1 ? NSA - 2 : 1) + E < 64, "vmcnt immediate");
  __shared__ __attribute__((aligned(16))) char smem[NSA * A_ST + 2 * B_ST];
  char* const sA = smem;
  char* const sB = smem + NSA * A_ST;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int nk = K / 64;
  int first, stride, limit = n_tiles;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    first = (int)((int64_t)n_tiles * xcd / 8) + (blockIdx.x >> 3);
    limit = (int)((int64_t)n_tiles * (xcd + 1) / 8);
    stride = gridDim.x >> 3;
  } else {
    first = blockIdx.x;
    stride = gridDim.x;
  }
  const int n_mine = first < limit ? (limit - first + stride - 1) / stride : 0;
  const int S = n_mine * nk;
  if (S == 0) return;

  // per-lane source byte offsets (row 8 j + lane / 8, swizzled chunk) of this wave's pieces
  int voa[PA], vob[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int row = 8 * (wave * PA + p) + (lane >> 3);
    voa[p] = row * (int)(lda * 2) + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int row = 8 * (wave * PB + p) + (lane >> 3);
    vob[p] = row * (int)(ldb * 2) + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // A and B DMA positions advance separately (A runs NSA - 2 K-steps further ahead)
  __amdgpu_buffer_rsrc_t ra, rb;
  auto rsrc_a = [&](int i) {
    const int tile = first + i * stride, tm = tile / tiles_n, m0 = tm * MT;
    ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(A + (int64_t)m0 * lda), (short)0,
                                           (int)min((int64_t)(M - m0) * lda * 2, (int64_t)0x7ffffff0), 0x00020000);
  };
  auto rsrc_b = [&](int i) {
    const int tile = first + i * stride, tm = tile / tiles_n, n0 = (tile - tm * tiles_n) * BN;
    rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(B + (int64_t)n0 * ldb), (short)0,
                                           (int)min((int64_t)BN * ldb * 2, (int64_t)0x7ffffff0), 0x00020000);
  };
  auto dma_a = [&](int st, int p, int kt) {
#if MMT_W384_ABL != 2
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        ra, (__attribute__((address_space(3))) void*)(sA + st * A_ST + (wave * PA + p) * 1024), 16,
        voa[p], kt * 128, 0, 0);
#endif
  };
  auto dma_b = [&](int st, int p, int kt) {
#if MMT_W384_ABL != 2 && MMT_W384_ABL != 1
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rb, (__attribute__((address_space(3))) void*)(sB + st * B_ST + (wave * PB + p) * 1024), 16,
        vob[p], kt * 128, 0, 0);
#endif
  };
#else
  auto rsrc_a = [&](int) {};
  auto rsrc_b = [&](int) {};
  auto dma_a = [&](int, int, int) {};
  auto dma_b = [&](int, int, int) {};
#endif
  int ai = 0, akt = 0, as = 0;  // next A K-step to load: tile index, K-step, sequence number
  int bi = 0, bkt = 0, bs = 0;  // next B K-step to load
  rsrc_a(0);
  rsrc_b(0);
  auto next_a = [&]() {
    ++as;
    if (++akt == nk) {
      akt = 0;
      if (++ai < n_mine) rsrc_a(ai);
    }
  };
  auto next_b = [&]() {
    ++bs;
    if (++bkt == nk) {
      bkt = 0;
      if (++bi < n_mine) rsrc_b(bi);
    }
  };

  floatx16 acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int l31 = lane & 31, h = lane >> 5;
  int a_off[MB], b_off[NB];  // fragment row byte offsets; the rows' swizzle is (l31 >> 1) & 7
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) a_off[mb] = (wm * WM + 32 * mb + l31) * 128;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) b_off[nb] = (wn * 96 + 32 * nb + l31) * 128;
  const int sw = (l31 >> 1) & 7;

  // the K-step in A stage sta / B stage stb; the DMA of the next B K-step and of the A K-step
  // NSA - 1 ahead (in that order) goes between the MFMA groups, so the SIMD partner wave keeps
  // issuing MFMAs while this one issues DMA
  constexpr int PP = PA + PB;
  auto compute = [&](int sta, int stb, bool nb_ok, bool na_ok) {
    const char* SA = sA + sta * A_ST;
    const char* SB = sB + stb * B_ST;
    const int nbs = bs & 1, nas = as % NSA;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = ((2 * ks + h) ^ sw) << 4;
      bf16x8 af[MB], bfr[NB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) af[mb] = *reinterpret_cast<const bf16x8*>(SA + a_off[mb] + c);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) bfr[nb] = *reinterpret_cast<const bf16x8*>(SB + b_off[nb] + c);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#if MMT_W384_ABL == 3
          if (M < 0)
#endif
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[nb], af[mb], acc[mb][nb], 0, 0, 0);
        const int g = ks * MB + mb;  // DMA pieces over the (ks, mb) MFMA groups: B first, then A
        if (g < PB) {
          if (nb_ok) dma_b(nbs, g, bkt);
        } else if (g < PP) {
          if (na_ok) dma_a(nas, g - PB, akt);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int g = 4 * MB; g < PP; ++g) {
      if (g < PB) {
        if (nb_ok) dma_b(nbs, g, bkt);
      } else {
        if (na_ok) dma_a(nas, g - PB, akt);
      }
    }
  };

  // lane (row l31, half h) holds, per 32-column block, columns 8 g + 4 h + i (acc[4 g + i]);
  // v_permlane32_swap of the g = 2 j and 2 j + 1 runs gives it 8 contiguous columns
  // 16 j + 8 h .. + 7
  auto epilogue = [&](int tile) {
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int gr = tm * MT + wm * WM + 32 * mb + l31;
      const bool ok = gr < M;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[mb][nb][8 * j + i]),
                                                            __float_as_uint(acc[mb][nb][8 * j + 4 + i]),
                                                            false, false);
            v[i] = __uint_as_float(x[0]);
            v[4 + i] = __uint_as_float(x[1]);
          }
          const int gc = tn * BN + wn * 96 + 32 * nb + 16 * j + 8 * h;
          if constexpr (EP == 1) {
            const uint4 u = *reinterpret_cast<const uint4*>(R + (int64_t)(ok ? gr : M - 1) * ldr + gc);
            const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[2 * q] += __uint_as_float(w[q] << 16);
              v[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
            }
          }
          if constexpr (EP == 2)
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
          uint4 o;
          o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
          o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
          if (ok) *reinterpret_cast<uint4*>(C + (int64_t)gr * ldc + gc) = o;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mb][nb][r] = 0.f;
      }
    }
  };

  // prologue, issue order B(0), A(0) .. A(NSA - 2)
#pragma unroll
  for (int p = 0; p < PB; ++p) dma_b(0, p, bkt);
  next_b();
#pragma unroll
  for (int q = 0; q < NSA - 1; ++q)
    if (q < S) {
#pragma unroll
      for (int p = 0; p < PA; ++p) dma_a(q, p, akt);
      next_a();
    }
  bool stored = false;  // the previous K-step ended a full tile: its E stores are the youngest
  int i = 0, kt = 0;    // the computed K-step's tile and K-step
  for (int s = 0; s < S; ++s) {
    // K-step s needs B(s) and A(s). Younger than B(s): for s = 0 the prologue's A(1 ..
    // NSA - 2), otherwise A(s + NSA - 2) (issued right after it, if it exists) and the stores
    // of an epilogue at the end of K-step s - 1.
    // (with NSA = 2, A(s + NSA - 2) is A(s) itself: nothing may stay in flight)
    const int ya = s == 0 ? min(NSA - 2, S - 1) : (NSA >= 3 && s + NSA - 2 < S ? 1 : 0);
    if (ya == 0) {
      if (stored) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(E) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (ya == 1) {
      if (stored) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PA + E) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PA) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PA * (NSA - 2 > 1 ? NSA - 2 : 1)) : "memory");
    }
    asm volatile("s_barrier" ::: "memory");  // K-step s landed for every wave; its predecessor's stages free
    const bool nb_ok = bs < S, na_ok = as < S;
    compute(s % NSA, s & 1, nb_ok, na_ok);
    if (nb_ok) next_b();
    if (na_ok) next_a();
    stored = false;
    if (++kt == nk) {
      const int tile = first + i * stride;
      epilogue(tile);
      stored = EP != 1 && (tile / tiles_n) * MT + MT <= M;
      kt = 0;
      ++i;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Weight-gradient (TN) split-K partial products with direct global->LDS loads: slab[z] =
// A[k0:k1]^T . B[k0:k1] for A [K][M] (dY, rows = tokens) and B [K][N] (X), both MN-contiguous.
// 256 x 192 output tile, 8 waves as 4 (M) x 2 (N) of 64 x 96 (2 x 3 MFMA 32x32x16 blocks, the
// register-staged gemm_big_kernel's geometry), K-steps of 64 tokens, two LDS stages of unpadded
// [64][256] + [64][192] bf16 images (56 KB each) filled by buffer_load ... lds (no VGPR staging,
// no ds_write pass: the register-staged kernel spent 56 KB of ds_write per K-step on top of the
// fragment reads). The 16-B chunk c of k-row r sits at c ^ swA/swB(r) (applied to each lane's
// SOURCE address, the DMA destination is lane-linear), so each 32-lane group of a transposed
// fragment read (ds_read_b64_tr_b16: 4 k-rows x 64 B) covers the 64 banks once.
// Columns past M / N read whatever lies there (only output rows / columns past M / N depend on
// them, and those are not stored); rows past K read zeros (buffer range). One tile per workgroup,
// so the K-loop carries no stores: the wait for a K-step's DMA is vmcnt(0) on nothing else.
constexpr int TN_BM = 256, TN_BN = 192, TN_NT = 512;
#ifndef MMT_TN_ABL  // ablation / variant builds (tools/build_abl_tn.sh)
#define MMT_TN_ABL 0
#endif
// buffer_load_dwordx4 ... lds as inline asm (same operation as dma16): issued through the
// builtin, the compiler cannot tell the transposed fragment reads (ds_read_b64_tr_b16) from the
// stage being filled and puts a vmcnt(0) behind every DMA (the next K-step's, meant to stay in
// flight under these MFMAs). Completion is waited for explicitly (vmcnt(0) + s_barrier at the
// top of each K-step). dma16_asm: common.h.
// BM: tile height, 256 (8 waves of 64 x 96: 2 x 3 MFMA blocks) or 384 (waves of 96 x 96: 3 x 3
// blocks; 72 KB per K-step for 1.5x the products of the 56 KB 256-row step — the kernel is bound
// by its DMA rate, profiles/r03_tn_ablation.txt).
template <int BM>
__global__ __launch_bounds__(TN_NT, 1) void gemm_tn_dma_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
    int64_t ldb, float* __restrict__ slab, int split_k, int k_chunk, int tiles_n) {
  static_assert(BM == 256 || BM == 384, "tile height");
  constexpr int MB = BM / 128;                                      // 32-row MFMA blocks per wave
  constexpr int A_ROWB = BM * 2, B_ROWB = TN_BN * 2;                // bytes per k-row
  constexpr int A_CH = A_ROWB / 16;                                 // 16-B chunks per A k-row
  constexpr int A_BYTES = 64 * A_ROWB, B_BYTES = 64 * B_ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int GA = A_BYTES / 1024 / 8, GB = B_BYTES / 1024 / 8;   // DMA pieces per wave (4 / 6 + 3)
  constexpr int G = GA + GB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1, hl = lane >> 5;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int wi = xcd_remap(blockIdx.x, gridDim.x);
  const int z = wi / tiles, t = wi - z * tiles;
  const int tm = t / tiles_n;
  const int m0 = tm * BM, n0 = (t - tm * tiles_n) * TN_BN;
  const int kbeg = z * k_chunk, kend = min(K, kbeg + k_chunk);
  const int nk = max(0, (kend - kbeg + 63) / 64);
  // chunk swizzles (16-B chunks of a k-row): A rows are 512 B (every row starts on bank 0), so
  // the 4 k-rows of a transposed read take 4 disjoint 64-B slots: c ^ 4 (r & 3); B rows are
  // 384 B (odd rows start half a bank window on), c ^ 2 (r & 3) keeps them apart (simulated for
  // every fragment read; the A form 2 (r & 3) measured 29 % of LDS cycles in bank conflicts)
  auto swA = [](int r) { return 4 * (r & 3); };
  auto swB = [](int r) { return 2 * (r & 3); };

  // per-lane source offsets (bytes from the K-step's panel base) of this wave's DMA pieces
  int voff[G];
#pragma unroll
  for (int p = 0; p < G; ++p) {
    if (p < GA) {  // A piece j = wave * GA + p: 1 KB of the [64][BM] image (A_CH chunks per k-row;
                   // 768-B rows also start on bank 0: the same swizzle)
      const int j = wave * GA + p, e = j * 64 + lane, row = e / A_CH, c = (e % A_CH) ^ swA(row);
      voff[p] = row * (int)(lda * 2) + c * 16;
    } else {       // B piece j: 1 KB of the [64][192] image (24 chunks per k-row)
      const int j = wave * GB + (p - GA), e = j * 64 + lane, row = e / 24, c = (e % 24) ^ swB(row);
      voff[p] = row * (int)(ldb * 2) + c * 16;
    }
  }
  // buffer ranges end at row K (zeros past it); the panel base moves with the K-step
  auto piece = [&](int kt, int st, int p) {
#if MMT_TN_ABL == 1 || MMT_TN_ABL == 4  // ablation builds (tools/build_abl_tn.sh): no DMA
    if (K > 0) return;
#endif
#if MMT_TN_ABL == 6  // ablation: B pieces only
    if (p < GA) return;
#endif
#if MMT_TN_ABL == 7  // ablation: A pieces only
    if (p >= GA) return;
#endif
#if MMT_TN_ABL == 5  // ablation: every split reads the first K chunk (L2-shared)
    const int k0 = kt * 64;
#else
    const int k0 = kbeg + kt * 64;
#endif
    char* S0 = smem + st * STAGE;
    if (p < GA)
      dma16_asm(A + (int64_t)k0 * lda + m0, ((int64_t)(K - k0) * lda - m0) * 2,
                S0 + (wave * GA + p) * 1024, voff[p]);
    else
      dma16_asm(B + (int64_t)k0 * ldb + n0, ((int64_t)(K - k0) * ldb - n0) * 2,
                S0 + A_BYTES + (wave * GB + (p - GA)) * 1024, voff[p]);
  };

  floatx16 acc[MB][3];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;

  // fragment of rows rbase.. (M or N index) for k-slice ks: lane (i = lane & 15: k-row q = i >> 2,
  // column group p4 = i & 3; g = lane >> 4; h = lane >> 5) reads 4 columns of k-rows k1 and k1 + 4
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g16 = lane >> 4;
  auto frag = [&](const char* S, int rowb, int rbase, int ks) {
    const int col = rbase + 16 * (g16 & 1) + 4 * p4;
    const int k1 = ks * 16 + 8 * hl + q4;
    const int cofs = (col & 7) * 2;
    const int s1 = rowb == A_ROWB ? swA(k1) : swB(k1);
    const int s2 = rowb == A_ROWB ? swA(k1 + 4) : swB(k1 + 4);
    const short4v v1 = tr_read(reinterpret_cast<const bf16_t*>(
        S + k1 * rowb + ((((col >> 3) ^ s1)) << 4) + cofs));
    const short4v v2 = tr_read(reinterpret_cast<const bf16_t*>(
        S + (k1 + 4) * rowb + ((((col >> 3) ^ s2)) << 4) + cofs));
    short __attribute__((ext_vector_type(8))) v = {v1[0], v1[1], v1[2], v1[3],
                                                   v2[0], v2[1], v2[2], v2[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  if (nk > 0)
#pragma unroll
    for (int p = 0; p < G; ++p) piece(0, 0, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    // this K-step's DMA is the only memory operation in flight
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const bool nxt = kt + 1 < nk;
    const char* As = smem + st * STAGE;
    const char* Bs = As + A_BYTES;
    // the next K-step's DMA into the other stage (free since this barrier), all of it before any
    // MFMA so every piece has the whole K-step to land (spread over the k-slices, the last pieces
    // were issued just before the next barrier's wait): interleaved on one box
    // (tools/gpu_wgrad_ab2.sh) MLP Dense_0 dW 187-190 -> 181-183 us, QKV 158 -> 152-153 us,
    // Dense_1 191-194 -> 183-184 us; step 15,924 -> 15,970 samples/s
    if (nxt)
#pragma unroll
      for (int p = 0; p < G; ++p) piece(kt + 1, st ^ 1, p);
    // fragments one k-slice ahead: slice ks + 1's reads are in flight under slice ks's MFMAs (every
    // wave reaches this point together after the barrier, so the partner wave cannot cover them)
    bf16x8 af[2][MB], bfr[2][3];
#pragma unroll
    for (int a = 0; a < MB; ++a) af[0][a] = frag(As, A_ROWB, wm * (32 * MB) + a * 32, 0);
#pragma unroll
    for (int b = 0; b < 3; ++b) bfr[0][b] = frag(Bs, B_ROWB, wn * 96 + b * 32, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int cu = ks & 1;
#if MMT_TN_ABL == 3 || MMT_TN_ABL == 4  // ablation: fragments of k-slice 0 reused (no further reads)
      if (ks < 3 && K < 0) {
#else
      if (ks < 3) {
#endif
#pragma unroll
        for (int a = 0; a < MB; ++a) af[cu ^ 1][a] = frag(As, A_ROWB, wm * (32 * MB) + a * 32, ks + 1);
#pragma unroll
        for (int b = 0; b < 3; ++b) bfr[cu ^ 1][b] = frag(Bs, B_ROWB, wn * 96 + b * 32, ks + 1);
      }
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b)  // operands swapped: the accumulator holds C^T
#if MMT_TN_ABL == 2  // ablation: no MFMAs (fragments kept live)
          asm volatile("" ::"v"(bfr[cu][b]), "v"(af[cu][a]));
#else
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[cu][b], af[cu][a], acc[a][b], 0, 0, 0);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // fp32 slab z: lane (m = lane & 31, h) of block (a, b) holds row m, columns 8g + 4h + {0..3}
  float* out = slab + (int64_t)z * M * N;
#pragma unroll
  for (int a = 0; a < MB; ++a) {
    const int gr = m0 + wm * (32 * MB) + a * 32 + (lane & 31);
    if (gr >= M) continue;
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int gc = n0 + wn * 96 + b * 32 + 8 * g + 4 * hl;
        if (gc >= N) continue;
        *reinterpret_cast<float4*>(out + (int64_t)gr * N + gc) =
            make_float4(acc[a][b][4 * g], acc[a][b][4 * g + 1], acc[a][b][4 * g + 2],
                        acc[a][b][4 * g + 3]);
      }
  }
}

// ---------------------------------------------------------------------------------------------
// The two-stage TN kernel above on v_mfma_f32_16x16x32_bf16 (round 5): the same tile, K-steps,
// DMA and wave grid, but 6 x 6 blocks of 16 x 16 per 96 x 96 wave tile and k32 MFMA steps (the
// same LDS bytes and MFMA cycles per K-step; MI355X_MICROARCH.md "DVFS give-back" item 7: the chip
// holds a higher clock on the 16x16 shape, 1.12-1.15x the FLOP/s of 32x32x16 with operands re-read
// from LDS). A 16x16x32 fragment reads k-rows k1 + 8 g (g = lane >> 4 in 0..3): rows r and r + 8
// of one read instruction, so the chunk swizzles also XOR bit 3 of the k-row (swA16 / swB16:
// conflict-free for both fragment shapes). Per k32 step the B fragments are consumed b-outer, so
// each B register set is refilled with the next step's fragment as soon as its 6 MFMAs issued
// (one A set in flight ahead, B refilled in place: 216 registers). Results agree with the 32x32
// kernels to fp32 rounding (different k grouping inside the MFMA), not bit for bit.
template <int V>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(V) : "memory");
}
// s_waitcnt vmcnt(y * C) for a runtime y in [0, Y] (y == Y, the steady state, tested first)
template <int C, int Y>
__device__ __forceinline__ void vm_wait_slices(int y) {
  if constexpr (Y <= 0) {
    vm_wait_n<0>();
  } else {
    if (y >= Y) vm_wait_n<Y * C>();
    else vm_wait_slices<C, Y - 1>(y);
  }
}
typedef float f32x4_t __attribute__((ext_vector_type(4)));
template <int BM>
__global__ __launch_bounds__(TN_NT, 1) void gemm_tn_dma16_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
    int64_t ldb, float* __restrict__ slab, int split_k, int k_chunk, int tiles_n) {
  static_assert(BM == 256 || BM == 384, "tile height");
  constexpr int MA = BM / 64;                                       // 16-row A blocks per wave
  constexpr int A_ROWB = BM * 2, B_ROWB = TN_BN * 2;
  constexpr int A_CH = A_ROWB / 16;
  constexpr int A_BYTES = 64 * A_ROWB, B_BYTES = 64 * B_ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int GA = A_BYTES / 1024 / 8, GB = B_BYTES / 1024 / 8;
  constexpr int G = GA + GB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int wi = xcd_remap(blockIdx.x, gridDim.x);
  const int z = wi / tiles, t = wi - z * tiles;
  const int tm = t / tiles_n;
  const int m0 = tm * BM, n0 = (t - tm * tiles_n) * TN_BN;
  const int kbeg = z * k_chunk, kend = min(K, kbeg + k_chunk);
  const int nk = max(0, (kend - kbeg + 63) / 64);
  auto swA = [](int r) { return (4 * (r & 3)) ^ (2 * ((r >> 3) & 1)); };
  auto swB = [](int r) { return (2 * (r & 3)) ^ (2 * ((r >> 3) & 1)); };
  int voff[G];
#pragma unroll
  for (int p = 0; p < G; ++p) {
    if (p < GA) {
      const int j = wave * GA + p, e = j * 64 + lane, row = e / A_CH, c = (e % A_CH) ^ swA(row);
      voff[p] = row * (int)(lda * 2) + c * 16;
    } else {
      const int j = wave * GB + (p - GA), e = j * 64 + lane, row = e / 24, c = (e % 24) ^ swB(row);
      voff[p] = row * (int)(ldb * 2) + c * 16;
    }
  }
  auto piece = [&](int kt, int st, int p) {
    const int k0 = kbeg + kt * 64;
    char* S0 = smem + st * STAGE;
    if (p < GA)
      dma16_asm(A + (int64_t)k0 * lda + m0, ((int64_t)(K - k0) * lda - m0) * 2,
                S0 + (wave * GA + p) * 1024, voff[p]);
    else
      dma16_asm(B + (int64_t)k0 * ldb + n0, ((int64_t)(K - k0) * ldb - n0) * 2,
                S0 + A_BYTES + (wave * GB + (p - GA)) * 1024, voff[p]);
  };
  f32x4_t acc[MA][6];
#pragma unroll
  for (int a = 0; a < MA; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[a][b][q] = 0.f;
  // 16x16x32 fragment of rows rbase.. for k32 step ks: lane (i = lane & 15: k-row q = i >> 2,
  // column group p4 = i & 3; g = lane >> 4) reads 4 columns of k-rows 32 ks + 8 g + q and + 4
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g16 = lane >> 4;
  auto frag = [&](const char* S, int rowb, int rbase, int ks) {
    const int col = rbase + 4 * p4;
    const int k1 = ks * 32 + 8 * g16 + q4;
    const int cofs = (col & 7) * 2;
    const int s1 = rowb == A_ROWB ? swA(k1) : swB(k1);
    const int s2 = rowb == A_ROWB ? swA(k1 + 4) : swB(k1 + 4);
    const short4v v1 = tr_read(reinterpret_cast<const bf16_t*>(
        S + k1 * rowb + ((((col >> 3) ^ s1)) << 4) + cofs));
    const short4v v2 = tr_read(reinterpret_cast<const bf16_t*>(
        S + (k1 + 4) * rowb + ((((col >> 3) ^ s2)) << 4) + cofs));
    short __attribute__((ext_vector_type(8))) v = {v1[0], v1[1], v1[2], v1[3],
                                                   v2[0], v2[1], v2[2], v2[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  if (nk > 0)
#pragma unroll
    for (int p = 0; p < G; ++p) piece(0, 0, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const char* As = smem + st * STAGE;
    const char* Bs = As + A_BYTES;
    if (kt + 1 < nk)
#pragma unroll
      for (int p = 0; p < G; ++p) piece(kt + 1, st ^ 1, p);
    bf16x8 af[2][MA], bfr[6];
#pragma unroll
    for (int a = 0; a < MA; ++a) af[0][a] = frag(As, A_ROWB, wm * (16 * MA) + a * 16, 0);
#pragma unroll
    for (int b = 0; b < 6; ++b) bfr[b] = frag(Bs, B_ROWB, wn * 96 + b * 16, 0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks == 0)
#pragma unroll
        for (int a = 0; a < MA; ++a) af[1][a] = frag(As, A_ROWB, wm * (16 * MA) + a * 16, 1);
#pragma unroll
      for (int b = 0; b < 6; ++b) {
#pragma unroll
        for (int a = 0; a < MA; ++a)  // operands swapped: the accumulator holds C^T
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[ks][a], acc[a][b], 0, 0, 0);
        if (ks == 0) bfr[b] = frag(Bs, B_ROWB, wn * 96 + b * 16, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // fp32 slab z: lane (m = lane & 15, g) of block (a, b) holds row m, columns 4 g + {0..3}
  float* out = slab + (int64_t)z * M * N;
#pragma unroll
  for (int a = 0; a < MA; ++a) {
    const int gr = m0 + wm * (16 * MA) + a * 16 + (lane & 15);
    if (gr >= M) continue;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int gc = n0 + wn * 96 + b * 16 + 4 * g16;
      if (gc >= N) continue;
      *reinterpret_cast<float4*>(out + (int64_t)gr * N + gc) =
          make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// TN weight gradients on a FOUR-STAGE RING of 32-row K-steps (round 5): gemm_tn_dma16_kernel's
// tile, wave grid, swizzles, 16x16x32 MFMAs and k order (the slabs are bit-identical), but the LDS
// holds four K-steps of 32 k-rows (36 KB each at BM 384, 144 KB) and the DMA runs three K-steps
// ahead of the one whose MFMAs issue. The fill pattern alone (tools/dma_lab.hip, the Dense_0 dW
// grid) takes 142 us through the two-stage kernel's wait-all + barrier per 64 rows and 117 us
// through this ring (profiles/r05_dma_lab.txt): the two-stage structure, not the HBM, set the
// K-step rate. Per K-step s, after one s_barrier (every wave's DMA of step s + 1 landed, every
// wave's fragment reads of step s done):
//   * the DMA of step s + 4 goes into step s's slot (its fragments are in registers),
//   * 36 MFMAs consume step s's fragments while step s + 1's are read into the other A set and,
//     B-outer, into each B register as soon as its 6 MFMAs issued (the dma16 kernel's k32 overlap
//     carried across K-steps, so every fragment read sits under MFMAs).
// The 36 1-KB pieces of a step are dealt 3 A + 2 B to waves 0-3 and 3 A + 1 B to waves 4-7, each
// wave waiting vmcnt(y x its own piece count) for the younger steps.
template <int BM>
__global__ __launch_bounds__(TN_NT, 1) void gemm_tn_r4_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
    int64_t ldb, float* __restrict__ slab, int split_k, int k_chunk, int tiles_n) {
  static_assert(BM == 384, "tile height");
  constexpr int MA = BM / 64;                                       // 16-row A blocks per wave
  constexpr int SK = 32, NS = 4;                                    // k-rows per step, slots
  constexpr int A_ROWB = BM * 2, B_ROWB = TN_BN * 2;
  constexpr int A_CH = A_ROWB / 16;
  constexpr int A_BYTES = SK * A_ROWB, B_BYTES = SK * B_ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = A_BYTES / 1024, PB = B_BYTES / 1024;           // 24 + 12 pieces
  static_assert(PA == 24 && PB == 12, "piece deal");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int wi = xcd_remap(blockIdx.x, gridDim.x);
  const int z = wi / tiles, t = wi - z * tiles;
  const int tm = t / tiles_n;
  const int m0 = tm * BM, n0 = (t - tm * tiles_n) * TN_BN;
  const int kbeg = z * k_chunk, kend = min(K, kbeg + k_chunk);
  const int nk = max(0, (kend - kbeg + SK - 1) / SK);
  auto swA = [](int r) { return (4 * (r & 3)) ^ (2 * ((r >> 3) & 1)); };
  auto swB = [](int r) { return (2 * (r & 3)) ^ (2 * ((r >> 3) & 1)); };
  const bool big = wave < 4;                                        // 5 pieces (else 4)
  int voff[5], ldso[5];
#pragma unroll
  for (int p = 0; p < 5; ++p) {
    if (p < 3) {
      const int j = wave * 3 + p, e = j * 64 + lane, row = e / A_CH, c = (e % A_CH) ^ swA(row);
      voff[p] = row * (int)(lda * 2) + c * 16;
      ldso[p] = j * 1024;
    } else {
      const int j = min(wave + 8 * (p - 3), PB - 1);
      const int e = j * 64 + lane, row = e / 24, c = (e % 24) ^ swB(row);
      voff[p] = row * (int)(ldb * 2) + c * 16;
      ldso[p] = A_BYTES + j * 1024;
    }
  }
  // piece p of step s (p < 3: A, else B; p == 4 only on the big waves)
  auto piece = [&](int s, int p) {
    const int k0 = kbeg + s * SK;
    char* S0 = smem + (s % NS) * STAGE;
    if (p < 3)
      dma16_asm(A + (int64_t)k0 * lda + m0, ((int64_t)(K - k0) * lda - m0) * 2, S0 + ldso[p], voff[p]);
    else if (p == 3 || big)
      dma16_asm(B + (int64_t)k0 * ldb + n0, ((int64_t)(K - k0) * ldb - n0) * 2, S0 + ldso[p], voff[p]);
  };
  auto issue = [&](int s) {  // (issued between the MFMA groups instead: 7 % slower)
#pragma unroll
    for (int p = 0; p < 5; ++p) piece(s, p);
  };
  // wait until this wave's pieces of every step older than the y youngest issued have landed
  auto wait_steps = [&](int y) {
    if (big) vm_wait_slices<5, 3>(y);
    else vm_wait_slices<4, 3>(y);
  };
  f32x4_t acc[MA][6];
#pragma unroll
  for (int a = 0; a < MA; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[a][b][q] = 0.f;
  const int i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3, g16 = lane >> 4;
  auto frag = [&](const char* S, int rowb, int rbase) {
    const int col = rbase + 4 * p4;
    const int k1 = 8 * g16 + q4;
    const int cofs = (col & 7) * 2;
    const int s1 = rowb == A_ROWB ? swA(k1) : swB(k1);
    const int s2 = rowb == A_ROWB ? swA(k1 + 4) : swB(k1 + 4);
    const short4v v1 = tr_read(reinterpret_cast<const bf16_t*>(
        S + k1 * rowb + ((((col >> 3) ^ s1)) << 4) + cofs));
    const short4v v2 = tr_read(reinterpret_cast<const bf16_t*>(
        S + (k1 + 4) * rowb + ((((col >> 3) ^ s2)) << 4) + cofs));
    short __attribute__((ext_vector_type(8))) v = {v1[0], v1[1], v1[2], v1[3],
                                                   v2[0], v2[1], v2[2], v2[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  bf16x8 af0[MA], af1[MA], bfr[6];
  // one K-step: wait for step s + 1, barrier, refill slot s, MFMAs on s with s + 1's reads under them
  auto body = [&](int s, bf16x8 (&ca)[MA], bf16x8 (&na)[MA]) {
    const bool nxt = s + 1 < nk;
    if (nxt) wait_steps(min(NS - 2, nk - 2 - s));
    // lgkmcnt(0) through the builtin (vmcnt / expcnt fields at their maxima): the compiler's own
    // wait insertion then knows every fragment read is retired and puts no lgkmcnt(0) in front of
    // the first MFMA (behind the next step's reads, as it did with the wait as inline asm)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");
    if (s + NS < nk) issue(s + NS);
    const char* As = smem + ((s + 1) % NS) * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
#pragma unroll
      for (int a = 0; a < MA; ++a)  // operands swapped: the accumulator holds C^T
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], ca[a], acc[a][b], 0, 0, 0);
      // the next step's A fragments behind the first B group's MFMAs (the last step reads a
      // stale slot: in bounds, never consumed)
      if (b == 0)
#pragma unroll
        for (int a = 0; a < MA; ++a) na[a] = frag(As, A_ROWB, wm * (16 * MA) + a * 16);
      bfr[b] = frag(Bs, B_ROWB, wn * 96 + b * 16);
      __builtin_amdgcn_sched_barrier(0);  // B refilled in place: no read hoisted above its MFMAs
    }
  };
#pragma unroll
  for (int q = 0; q < NS; ++q)
    if (q < nk) issue(q);
  if (nk > 0) {
    wait_steps(min(NS - 1, nk - 1));
    asm volatile("s_barrier" ::: "memory");
#pragma unroll
    for (int a = 0; a < MA; ++a) af0[a] = frag(smem, A_ROWB, wm * (16 * MA) + a * 16);
#pragma unroll
    for (int b = 0; b < 6; ++b) bfr[b] = frag(smem + A_BYTES, B_ROWB, wn * 96 + b * 16);
  }
  for (int s = 0; s < nk; s += 2) {
    body(s, af0, af1);
    if (s + 1 < nk) body(s + 1, af1, af0);
  }
  float* out = slab + (int64_t)z * M * N;
#pragma unroll
  for (int a = 0; a < MA; ++a) {
    const int gr = m0 + wm * (16 * MA) + a * 16 + (lane & 15);
    if (gr >= M) continue;
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int gc = n0 + wn * 96 + b * 16 + 4 * g16;
      if (gc >= N) continue;
      *reinterpret_cast<float4*>(out + (int64_t)gr * N + gc) =
          make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
    }
  }
}

// Split-K combine: v = sum_s slab[s][m][n] (fp32, slabs in order), then the GEMM epilogue, 4
// columns per thread with up to CB slabs' loads in flight (the slabs come from the Infinity
// Cache: the kernel is bound by loads in flight; 8 columns x 4 slabs per thread measured 37.6 us
// per launch in the step, 4 columns x 8 slabs less)
#ifndef MMT_COMBINE_CB  // slab loads in flight per thread (benchmarking builds)
#define MMT_COMBINE_CB 16
#endif
template <int OUT, int CB = MMT_COMBINE_CB>
__global__ void splitk_epilogue_kernel(const float* __restrict__ ws, int split, int M, int N,
                                       void* __restrict__ Cv, int64_t ldc, Epi epi) {
  const int n4 = N / 4;
  const int64_t total = (int64_t)M * n4;
  const int64_t slab = (int64_t)M * N;
  uint32_t key = 0;
  if (epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int gr = i / n4, gc = (i % n4) * 4;
    const float* p = ws + (int64_t)gr * N + gc;
    float v[4];
    ldw<4>(p, v);
    // slabs 1 .. split - 1 in batches of CB, every load of a batch issued before the first add
    // (predicated past split: no single-load tail), summed in slab order
    for (int k = 1; k < split; k += CB) {
      float t[CB][4];
#pragma unroll
      for (int j = 0; j < CB; ++j)
        if (k + j < split) ldw<4>(p + (k + j) * slab, t[j]);
#pragma unroll
      for (int j = 0; j < CB; ++j)
        if (k + j < split)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += t[j][e];
    }
    epilogue_w<4>(epi, key, N, gr, gc, v);
    store_w<OUT, 4>(Cv, (int64_t)gr * ldc + gc, epi.beta, v);
  }
}


// ---------------------------------------------------------------------------------------------
// Warp-specialised wide NT kernel (the bf16-output forward / gated products of the step: QKV,
// MLP up with bias + relu + dropout + relu_bits, the gated MLP input gradient with column sums).
// Why: in gemm_nt256_kernel every wave both issues the K-step DMA and stores its epilogue, and
// vmcnt retires loads and stores in one in-order counter, so the DMA wait after a tile's epilogue
// also waits for that epilogue's stores to be acknowledged (with every CU writing at once: K-steps
// 1.9 us instead of 1.04; the stores, not the MFMAs, set the pace of the K = 384 products). Here
// the roles are split by wave:
//  * waves 4-7 (loaders) issue every DMA piece (buffer_load ... lds, inline asm) and never store:
//    their vmcnt counts DMA only; three LDS stages, two K-steps in flight;
//  * waves 0-3 (one per SIMD) run the MFMAs and the epilogue; their stores are never waited for.
//    One s_barrier per K-step (all 8 waves): the loaders arrive after their K-step s DMA landed,
//    the compute waves after they finished reading K-step s - 1's stage (which the loaders refill
//    with K-step s + 2 right after the barrier).
// Tile 256 (M) x 128 (N): compute wave wm owns rows 64 wm .. + 63 and all 128 columns, with the
// per-wave fragment geometry, B-row permutation, swizzles and epilogue of nt256's BN = 256 wave
// (16x16x32 MFMA, operands swapped, lane = 4 rows x 32 columns in runs of 8): its outputs, its
// relu_bits / gate_bits words and its column sums are laid out exactly as nt256's (a 256-wide
// nt256 tile = two adjacent tiles here), and the column-sum slab is summed over the same 4 waves
// in the same order (bit-identical results).
// Requires !transA, transB, K % 64 == 0, N % 128 == 0, bf16 output, N <= WS_BIAS with a bias.
constexpr int WS_NT = 512, WS_BIAS = 2048;
template <bool CS, bool GBITS>
__global__ __launch_bounds__(WS_NT, 1) void gemm_ntws_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B,
    int64_t ldb, bf16_t* __restrict__ C, int64_t ldc, int tiles_n, int n_tiles, Epi epi) {
  constexpr int W = 128, NF = 8, Q = 32, NS = 3;
  constexpr int A_BYTES = 256 * 128, STAGE = A_BYTES + W * 128;  // 48 KB
  constexpr int PIECES = STAGE / 1024, PL = PIECES / 4;          // 48 pieces, 12 per loader
  constexpr int CS_FLOATS = CS ? 4 * W : 0;
  // ONE LDS object (a second one makes the compiler drain vmcnt before LDS reads)
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE + 4 * (WS_BIAS + CS_FLOATS)];
  float* const s_bias = reinterpret_cast<float*>(smem + NS * STAGE);
  float (*const s_cs)[W] = reinterpret_cast<float (*)[W]>(s_bias + WS_BIAS);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nk = K / 64;
  int first, stride, limit = n_tiles;
  if ((gridDim.x & 7) == 0) {  // each XCD a contiguous eighth of the row-panel-major tile list
    const int xcd = blockIdx.x & 7;
    first = (int)((int64_t)n_tiles * xcd / 8) + (blockIdx.x >> 3);
    limit = (int)((int64_t)n_tiles * (xcd + 1) / 8);
    stride = gridDim.x >> 3;
  } else {
    first = xcd_remap(blockIdx.x, gridDim.x);
    stride = gridDim.x;
  }
  const int n_mine = first < limit ? (limit - first + stride - 1) / stride : 0;
  const int S = n_mine * nk;
  if (S == 0) return;  // workgroup-uniform
  auto fA = [](int r) { return r & 6; };
  auto fB = [](int r) { return (r & 2) | (((r >> 3) & 1) << 2); };

  if (wave >= 4) {
    // ------------------------------------------------------------------ loader waves
    const int lw = wave - 4;
    // loader lw: A pieces 8 lw .. 8 lw + 7 (rows 8 j .. 8 j + 7 of the 256-row panel) and B pieces
    // 4 lw .. 4 lw + 3 (of the 128-row panel); the lane's 16-B chunk of its row at the row's
    // swizzle (source side; the LDS destination is lane-linear)
    constexpr int PLA = 8, PLB = 4;
    static_assert(PLA + PLB == PL, "pieces");
    int voa[PLA], vob[PLB];
#pragma unroll
    for (int i = 0; i < PLA; ++i) {
      const int row = 8 * (lw * PLA + i) + (lane >> 3);
      voa[i] = row * (int)(lda * 2) + (((lane & 7) ^ fA(row)) << 4);
    }
#pragma unroll
    for (int i = 0; i < PLB; ++i) {
      const int row = 8 * (lw * PLB + i) + (lane >> 3);
      vob[i] = row * (int)(ldb * 2) + (((lane & 7) ^ fB(row)) << 4);
    }
    auto issue = [&](int s) {  // K-step s of this workgroup's sequence into stage s % 3
      const int i = s / nk, kt = s - i * nk;
      const int tile = first + i * stride, tm = tile / tiles_n;
      const int m0 = tm * 256, n0 = (tile - tm * tiles_n) * W, k0 = kt * 64;
      char* S0 = smem + (s % NS) * STAGE;
      const bf16_t* pa = A + (int64_t)m0 * lda + k0;  // rows past M read zeros (buffer range)
      const int64_t ra = ((int64_t)(M - m0) * lda - k0) * 2;
      const bf16_t* pb = B + (int64_t)n0 * ldb + k0;
      const int64_t rb = ((int64_t)W * ldb - k0) * 2;
#pragma unroll
      for (int p = 0; p < PLA; ++p) dma16_asm(pa, ra, S0 + (lw * PLA + p) * 1024, voa[p]);
#pragma unroll
      for (int p = 0; p < PLB; ++p) dma16_asm(pb, rb, S0 + A_BYTES + (lw * PLB + p) * 1024, vob[p]);
    };
    issue(0);
    if (S > 1) issue(1);
    for (int s = 0; s < S; ++s) {
      // K-step s landed (K-step s + 1's pieces, issued after it, may stay in flight)
      if (s + 1 < S) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PL) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_barrier" ::: "memory");
      if (s + 2 < S) issue(s + 2);  // into the stage K-step s - 1 used (read before this barrier)
      if (CS && (s % nk) == nk - 1) asm volatile("s_barrier" ::: "memory");  // the tile's colsum sync
    }
    return;
  }

  // -------------------------------------------------------------------- compute waves
  const int wm = wave;
  if (epi.bias)  // N <= WS_BIAS (host); published by the loop's first barrier
    for (int i = threadIdx.x; i < N; i += 256) s_bias[i] = epi.bias[i];
  uint32_t key = 0;
  if (epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);
  Epi rest = epi;  // dropout / residual through epilogue_w; the rest inline (nt256 order)
  rest.alpha = 1.f;
  rest.bias = nullptr;
  rest.act = MMT_ACT_NONE;
  rest.gate = nullptr;
  rest.relu_bits = nullptr;
  rest.gate_bits = nullptr;
  constexpr bool RBITS = !CS && !GBITS;

  const int l15 = lane & 15, lq = lane >> 4;
  int a_off[4], a_sw[4], b_off[NF], b_sw[NF];
#pragma unroll
  for (int mf = 0; mf < 4; ++mf) {
    const int r = wm * 64 + mf * 16 + l15;
    a_off[mf] = r * 128;
    a_sw[mf] = fA(r);
  }
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int r = 32 * (nf >> 1) + 8 * (l15 >> 2) + 4 * (nf & 1) + (l15 & 3);
    b_off[nf] = A_BYTES + r * 128;
    b_sw[nf] = fB(r);
  }
  typedef float floatx4 __attribute__((ext_vector_type(4)));
  floatx4 acc[4][NF];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NF; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int st) {
    const char* S0 = smem + st * STAGE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 4 * h + lq;
      bf16x8 af[4], bfr[NF];
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
        af[mf] = *reinterpret_cast<const bf16x8*>(S0 + a_off[mf] + ((c ^ a_sw[mf]) << 4));
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
        bfr[nf] = *reinterpret_cast<const bf16x8*>(S0 + b_off[nf] + ((c ^ b_sw[nf]) << 4));
#pragma unroll
      for (int mf = 0; mf < 4; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nf], af[mf], acc[mf][nf], 0, 0, 0);
    }
  };

  // epilogue of `tile` (nt256's 256-wide epilogue for one wave, wn = 0, tile width 128); gbw: the
  // tile's gate_bits word, loaded at the tile's first K-step
  auto epilogue = [&](int tile, const uint4& gbw) {
    const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
    const int gc0 = tn * W + 8 * lq;
    float cs[CS ? Q : 1];
    if constexpr (CS)
#pragma unroll
      for (int j = 0; j < Q; ++j) cs[j] = 0.f;
    const int64_t bidx = (int64_t)(tm * 64 + wm * 16 + l15) * (N / 32) + (tn * 4 + lq);
    uint32_t rbw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int mf = 0; mf < 4; ++mf) {
      const int gr = tm * 256 + wm * 64 + mf * 16 + l15;
      if (gr < M) {
#pragma unroll
        for (int c8 = 0; c8 < Q / 8; ++c8) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = acc[mf][(8 * c8 + e) >> 2][e & 3] * epi.alpha;
          const int gc = gc0 + 32 * c8;
          if (epi.bias) {
            const float4 b0 = *reinterpret_cast<const float4*>(s_bias + gc);
            const float4 b1 = *reinterpret_cast<const float4*>(s_bias + gc + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
          }
          if (epi.act == MMT_ACT_RELU)
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
          if (GBITS) {
            const uint32_t w = (mf == 0 ? gbw.x : mf == 1 ? gbw.y : mf == 2 ? gbw.z : gbw.w) >> (8 * c8);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= ((w >> e) & 1u) ? epi.gate_scale : 0.f;
          }
          epilogue_w<8>(rest, key, N, gr, gc, v);
          if (RBITS && epi.relu_bits)
#pragma unroll
            for (int e = 0; e < 8; ++e) rbw[mf] |= (v[e] > 0.f ? 1u : 0u) << (8 * c8 + e);
          if constexpr (CS)
#pragma unroll
            for (int e = 0; e < 8; ++e) cs[8 * c8 + e] += __uint_as_float((uint32_t)f2bf(v[e]) << 16);
          store_w<0, 8>(C, (int64_t)gr * ldc + gc, 0.f, v);
        }
      }
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[mf][nf] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if (RBITS && epi.relu_bits)
      reinterpret_cast<uint4*>(epi.relu_bits)[bidx] = make_uint4(rbw[0], rbw[1], rbw[2], rbw[3]);
    if constexpr (CS) {
#pragma unroll
      for (int j = 0; j < Q; ++j) {  // sum over the 16 row lanes of each DPP row (as nt256)
        float x = cs[j];
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xf, 0xf, false));
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xf, 0xf, false));
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xf, 0xf, false));
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xf, 0xf, false));
        cs[j] = x;
      }
      if (l15 == 0)
#pragma unroll
        for (int j = 0; j < Q; ++j) s_cs[wm][32 * (j >> 3) + 8 * lq + (j & 7)] = cs[j];
      // the loaders meet this barrier after the tile's last K-step too (LDS only: no vmcnt)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (threadIdx.x < W)
        epi.colsum[(int64_t)tm * N + tn * W + threadIdx.x] =
            s_cs[0][threadIdx.x] + s_cs[1][threadIdx.x] + s_cs[2][threadIdx.x] + s_cs[3][threadIdx.x];
    }
  };

  uint4 gbw = make_uint4(0u, 0u, 0u, 0u);
  for (int s = 0; s < S; ++s) {
    const int i = s / nk, kt = s - i * nk;
    if (GBITS && kt == 0) {  // the tile's gate word, needed at its epilogue
      const int tile = first + i * stride, tm = tile / tiles_n, tn = tile - tm * tiles_n;
      gbw = reinterpret_cast<const uint4*>(epi.gate_bits)[(int64_t)(tm * 64 + wm * 16 + l15) * (N / 32) +
                                                          (tn * 4 + lq)];
    }
    // this wave's reads of K-step s - 1 are consumed (complete); LDS writes (bias) published
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    compute(s % NS);
    if (kt == nk - 1) epilogue(first + i * stride, gbw);
  }
}

// ---------------------------------------------------------------------------------------------
// FP8 (OCP e4m3) forward GEMM for the fp8 weight path (BASELINE configs[4]): C = epilogue(
// (A_q . B_q^T) * sa[m] * sb[n]) with A_q [M][K] e4m3 (activation rows quantised with one scale
// per row) and B_q [N][K] e4m3 (weight rows = output channels, one scale each). The products run
// on v_mfma_scale_f32_32x32x64_f8f6f4 with unit E8M0 block scales (the row / channel scales are
// applied exactly once in the epilogue, where they factor out of the K sum): twice the bf16 MFMA
// rate. Operands swapped (acc = C^T) so a lane holds one output row and four runs of 4 columns.
// Any consistent k order works for the MX operands (the hardware pairs byte j of lane half h of
// A with byte j of lane half h of B): lane (r, h) takes bytes 32h .. 32h+31 of its row's 64-byte
// K-step (tools/fp8_mfma_probe.hip checks the pairing with exact integers).
// 128 x 128 tiles, 4 waves as 2 x 2 of 64 x 64, K-steps of 64 bytes, double-buffered LDS rows
// padded to 80 bytes, register-staged loads one K-step ahead. Requires K % 64 == 0, N % 8 == 0.
constexpr int F8_BM = 128, F8_BN = 128, F8_RS = 80;
typedef int v8i __attribute__((ext_vector_type(8)));

template <int OUT>
__global__ __launch_bounds__(256, 2) void gemm_fp8_nt_kernel(
    int M, int N, int K, const uint8_t* __restrict__ A, int64_t lda, const float* __restrict__ sa,
    const uint8_t* __restrict__ B, int64_t ldb, const float* __restrict__ sb, void* __restrict__ Cv,
    int64_t ldc, int tiles_n, int n_work, Epi epi) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2][2][F8_BM * F8_RS];  // [stage][A | B]
  const int wi = xcd_remap(blockIdx.x, gridDim.x);
  if (wi >= n_work) return;
  const int tm = wi / tiles_n, tn = wi - tm * tiles_n;
  const int m0 = tm * F8_BM, n0 = tn * F8_BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  uint32_t key = 0;
  if (epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);
  // global -> register staging: 2 x 16 B of A and of B per thread per K-step (128 rows x 64 B)
  uint4 ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = threadIdx.x + 256 * q, row = c >> 2, ch = c & 3;
      ra[q] = *reinterpret_cast<const uint4*>(A + (int64_t)min(m0 + row, M - 1) * lda + k0 + 16 * ch);
      rb[q] = *reinterpret_cast<const uint4*>(B + (int64_t)min(n0 + row, N - 1) * ldb + k0 + 16 * ch);
    }
  };
  auto lstore = [&](int st) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c = threadIdx.x + 256 * q, row = c >> 2, ch = c & 3;
      const uint32_t ma = m0 + row < M ? 0xffffffffu : 0u;
      *reinterpret_cast<uint4*>(&smem[st][0][row * F8_RS + 16 * ch]) =
          make_uint4(ra[q].x & ma, ra[q].y & ma, ra[q].z & ma, ra[q].w & ma);
      *reinterpret_cast<uint4*>(&smem[st][1][row * F8_RS + 16 * ch]) = rb[q];
    }
  };
  typedef float floatx16_t __attribute__((ext_vector_type(16)));
  floatx16_t acc[2][2];  // [n sub-tile][m sub-tile]: C^T
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int nk = K / 64;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * 64);
    const uint8_t* As = smem[st][0];
    const uint8_t* Bs = smem[st][1];
    v8i xf[2], wf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint8_t* pa = As + (wm * 64 + 32 * t + (lane & 31)) * F8_RS + 32 * (lane >> 5);
      const uint8_t* pb = Bs + (wn * 64 + 32 * t + (lane & 31)) * F8_RS + 32 * (lane >> 5);
      const uint4 a0 = *reinterpret_cast<const uint4*>(pa), a1 = *reinterpret_cast<const uint4*>(pa + 16);
      const uint4 b0 = *reinterpret_cast<const uint4*>(pb), b1 = *reinterpret_cast<const uint4*>(pb + 16);
      xf[t] = v8i{(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
      wf[t] = v8i{(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(wf[a], xf[b], acc[a][b], 0, 0, 0,
                                                                     127, 0, 127);
    if (kt + 1 < nk) {
      // stage st^1 was last read in step kt-1, before the barrier that closed it
      lstore(st ^ 1);
      __syncthreads();
    }
  }
  // epilogue: lane = output row m; registers 4 g .. 4 g + 3 = columns n + 8 g + 4 h .. + 3
  const int hh = lane >> 5;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int gr = m0 + wm * 64 + 32 * b + (lane & 31);
    if (gr >= M) continue;
    const float s_row = sa[gr];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int gc = n0 + wn * 64 + 32 * a + 8 * g4 + 4 * hh;
        if (gc >= N) continue;
        float v[4];
        const float4 sw = *reinterpret_cast<const float4*>(sb + gc);
        v[0] = acc[a][b][4 * g4] * s_row * sw.x;
        v[1] = acc[a][b][4 * g4 + 1] * s_row * sw.y;
        v[2] = acc[a][b][4 * g4 + 2] * s_row * sw.z;
        v[3] = acc[a][b][4 * g4 + 3] * s_row * sw.w;
        epilogue_w<4>(epi, key, N, gr, gc, v);
        store_w<OUT, 4>(Cv, (int64_t)gr * ldc + gc, epi.beta, v);
      }
  }
}

// Row-wise e4m3 quantisation: scale[r] = amax(|x[r, :]|) / 448 (1 for an all-zero row),
// q[r, k] = e4m3(x[r, k] / scale[r]) with round-to-nearest-even (v_cvt_pk_fp8_f32, OCP).
// One wave per row; bf16 input rows with stride ld (16-B aligned), K % 8 == 0.
__global__ __launch_bounds__(256) void quant_rows_fp8_kernel(const bf16_t* __restrict__ x, int64_t ld,
                                                             int rows, int K, uint8_t* __restrict__ q,
                                                             int64_t ldq, float* __restrict__ scale) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bf16_t* xr = x + (int64_t)row * ld;
  float amax = 0.f;
  for (int k = lane * 8; k < K; k += 512) {
    const uint4 u = *reinterpret_cast<const uint4*>(xr + k);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      amax = fmaxf(amax, fmaxf(fabsf(__uint_as_float(w[e] << 16)), fabsf(__uint_as_float(w[e] & 0xffff0000u))));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  const float sc = amax > 0.f ? __fdiv_rn(amax, 448.f) : 1.f;
  if (lane == 0) scale[row] = sc;
  uint8_t* qr = q + (int64_t)row * ldq;
  for (int k = lane * 8; k < K; k += 512) {
    const uint4 u = *reinterpret_cast<const uint4*>(xr + k);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    uint32_t out[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float f0 = __fdiv_rn(__uint_as_float(w[2 * e] << 16), sc);
      const float f1 = __fdiv_rn(__uint_as_float(w[2 * e] & 0xffff0000u), sc);
      const float f2 = __fdiv_rn(__uint_as_float(w[2 * e + 1] << 16), sc);
      const float f3 = __fdiv_rn(__uint_as_float(w[2 * e + 1] & 0xffff0000u), sc);
      int pk = __builtin_amdgcn_cvt_pk_fp8_f32(f0, f1, 0, false);
      pk = __builtin_amdgcn_cvt_pk_fp8_f32(f2, f3, pk, true);
      out[e] = (uint32_t)pk;
    }
    *reinterpret_cast<uint2*>(qr + k) = make_uint2(out[0], out[1]);
  }
}

int cu_count() {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
      n_cu = 256;
  }
  return n_cu;
}

// Tile width of the persistent 256 x BN NT kernel for this launch, 0 when another kernel runs.
// the activation-stationary kernel (csrc/gemm_xs.hip) where it applies; MMT_XS=0: off (A/B)
int xs_mode() {  // 0 off, 1 bias-only bf16 products, 2 (default) also relu / dropout / relu bits
  static const int m = getenv("MMT_XS") ? atoi(getenv("MMT_XS")) : 2;
  return m;
}
bool xs_enabled() { return xs_mode() != 0; }

int nt_bn(int M, int N, int K, int transA, int transB, int batch, int out_kind, int final_kind) {
  if (transA || !transB || batch != 1 || out_kind == 2 || K % 64 != 0 ||
      !(g_variant < 0 || g_variant >= 5))
    return 0;
  const int tm256 = (M + 255) / 256;
  if (g_variant == 5) return N % 256 == 0 ? 256 : 0;
  if (g_variant == 6) return N % 192 == 0 ? 192 : 0;
  if (g_variant == 7) return N % 128 == 0 ? 128 : 0;
  // measured (tools/gemm_bench.py --variant=5/6/7 and gpu_exp/t5g.py, graph-timed): 256-wide
  // tiles at K <= 512 where N allows (MLP up 70656 x 1536 x 384: 125 us vs 141 at 192), 192-wide
  // otherwise (QKV 74752 x 1152 x 384; the T5 projections 8192 x 2304 / 3072 x 768: 45.9 / 50.2 us
  // vs 54.8 / 68.8 on the 128 x 128 kernels and 50.0 / 52.7 at 256); the narrow (N = 768 and
  // 384) and fp32 residual-stream shapes stay on the 128 x 128 kernels, faster there
  if (final_kind != 0 || N < 1152 || K > 768) return 0;
  const int bn = (K <= 512 && N % 256 == 0) ? 256 : N % 192 == 0 ? 192 : N % 256 == 0 ? 256 : 0;
  return bn && tm256 * (N / bn) >= cu_count() ? bn : 0;
}

// Whether the narrow-output NT kernel (gemm_ntw_kernel) runs this launch: products the library
// (hipBLASLt) used to take — narrow outputs over a long reduction (N <= 768, K >= 1152) and the
// bias-free relu product of the frozen T5 (N >= 2048, K <= 1024) — and the T5's plain QKV and
// o-projection products where they measured faster here; g_variant 8 forces it wherever it
// applies. Epilogues: none, bf16 residual, relu.
// MMT_NTWS (see mmt_gemm): 0 off, 1 the 192-wide-tile shapes, 2 every bf16 product it takes
int ntws_mode() {
  static const int m = getenv("MMT_NTWS") ? atoi(getenv("MMT_NTWS")) : 1;
  return m;
}

// The frozen T5's 768-wide bf16-residual products (o-projection, FF output) at 8192 < M <= 16384:
// nt256 with 192-wide tiles (measured, see ntw_ok)
bool t5_res768(int M, int N, const Epi& e) {
  return N == 768 && e.residual && !e.res_f32 && M > 8192 && M <= 16384 && g_variant < 0;
}

bool ntw_ok(int M, int N, int K, int transA, int transB, int batch, int out_kind, const Epi& e) {
  if (transA || !transB || batch != 1 || out_kind != 0 || N % 192 != 0 || K % 64 != 0) return false;
  if (e.bias || e.rng || e.gate || e.relu_bits || e.gate_bits || e.keep_bits || e.colsum || e.alpha != 1.f ||
      e.beta != 0.f || (e.residual && e.res_f32) || (e.residual && e.act != MMT_ACT_NONE) ||
      (e.act != MMT_ACT_NONE && e.act != MMT_ACT_RELU))
    return false;
  if (g_variant >= 0 && g_variant != 8) return false;
  if (g_variant == 8) return true;
  const bool narrow = N <= 768 && K >= 1152 && e.act == MMT_ACT_NONE;
  const bool relu = e.act == MMT_ACT_RELU && !e.residual && N >= 2048 && K <= 1024 && ntws_mode() != 2;
  // the frozen T5's other products at small batch (M = 32 B; tools/t5_small_probe.py, us per
  // launch, automatic choice vs this kernel): the plain QKV product 2304 x 768 at M 4096 / 8192
  // (30.1 / 46.9 vs 23.8 / 36.5), the o-projection + residual 768 x 768 at M 8192 (21.9 vs 20.4),
  // the relu product from M 4096 (28.9 vs 25.6). Round 6, at the bench batch (M = 16384,
  // tools/gpu_t5_variants.sh + tools/t5_products.py, this kernel with its conflict-free swizzle):
  // the QKV product 69.7 here vs 76.1 on nt256 (192-wide tiles); the two 768-wide residual
  // products faster on nt256's 192-wide tiles (t5_res768 below): o-projection 33.7 vs 36.0, FF
  // output 91.3 vs 97.8
  const bool wide_plain = e.act == MMT_ACT_NONE && !e.residual && N >= 2048 && K <= 1024;
  const bool square_res = e.residual && N == 768 && K <= 1024;
  if (t5_res768(M, N, e)) return false;
  return ((narrow || square_res) && M >= 8192) || (relu && M >= 4096) || (wide_plain && M >= 4096);
}

// Launch plan of gemm_ntw_kernel: tile width bn (192 / 384), `rows_big` rows in full rounds of
// the persistent grid on 256-row tiles, the rest on tiles of mt2 rows. A tile's time is taken as
// proportional to its operand bytes per K-step, (MT + BN) x 128, so a last round of a few big
// tiles is replaced by one of smaller tiles when that ends sooner.
struct NtwPlan {
  int bn, rows_big, mt2;
};
NtwPlan ntw_plan(int M, int N) {
  const int n_cu = cu_count();
  static const int force_mt = getenv("MMT_NTW_MT") ? atoi(getenv("MMT_NTW_MT")) : 0;  // tuning knobs
  static const int force_bn = getenv("MMT_NTW_BN") ? atoi(getenv("MMT_NTW_BN")) : 384;
  // 384-wide tiles (B re-read once per 256 rows) measured faster than 192-wide ones (A re-read
  // through L2 by two tiles, three A stages in flight): 204 vs 218 us at 138,496 x 384 x 1536
  const int bn = (force_bn == 192 || N % 384 != 0) ? 192 : 384;
  if (force_mt == 64 || force_mt == 128 || force_mt == 192 || force_mt == 256)
    if (bn == 384 || force_mt % 128 == 0) return {bn, 0, force_mt};
  const int tn = N / bn;
  const int panels_per_round = n_cu % tn == 0 ? n_cu / tn : 0;
  const int max_rounds = panels_per_round ? M / (256 * panels_per_round) : 0;
  NtwPlan best{bn, 0, 256};
  int64_t best_cost = INT64_MAX;
  for (int r = 0; r <= max_rounds; ++r) {
    const int rows_big = r * panels_per_round * 256, rem = M - rows_big;
    for (int mt : {64, 128, 192, 256}) {
      if (bn == 192 && mt % 128 != 0) continue;  // 4 x 2 waves of 32-row multiples
      const int64_t tiles = rem > 0 ? (int64_t)((rem + mt - 1) / mt) * tn : 0;
      const int64_t cost = (int64_t)r * (256 + bn) + ((tiles + n_cu - 1) / n_cu) * (mt + bn);
      if (cost < best_cost) {
        best_cost = cost;
        best = {bn, rows_big, mt};
      }
    }
  }
  return best;
}

// Dropout keeps of one (M, N) output in the relu_bits word layout (include/mmt_api.h): thread =
// one 16-B word group (4 rows x 32 columns), the same keep_elem draws the nt256 epilogue makes
// (pair counter ((row_offset + row) * N + col) / 2, 32-bit wrap included), so a launch that takes
// them as keep_bits stores bit-identical outputs. Pure VALU (64 mixer evaluations per thread, one
// 16-B store): it runs on a side queue beside attention.
__global__ __launch_bounds__(256) void dropout_keep_words_kernel(const uint32_t* __restrict__ rng,
                                                                 uint32_t layer, uint32_t site,
                                                                 uint32_t thresh16, int M, int N,
                                                                 int64_t row_off, uint4* __restrict__ out,
                                                                 int64_t n_words) {
  const uint32_t key = stream_key(rng[0], rng[1], layer, site);
  const int wpr = N / 32;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < n_words; idx += (int64_t)gridDim.x * 256) {
    const int64_t g = idx / wpr;
    const int w = (int)(idx - g * wpr);
    const int row0 = (int)(g >> 6) * 256 + (int)((g >> 4) & 3) * 64 + (int)(g & 15);
    const int col0 = 256 * (w >> 3) + 128 * ((w >> 2) & 1) + 8 * (w & 3);
    uint32_t o[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int r = row0 + 16 * f;
      uint32_t word = 0u;
      if (r < M) {
        const uint32_t base = (uint32_t)((row_off + r) * (int64_t)N + col0);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const uint32_t d = pair_draw(key, (base + 32 * c + e) >> 1);
            word |= ((d & 0xffffu) < thresh16 ? 1u : 0u) << (8 * c + e);
            word |= ((d >> 16) < thresh16 ? 1u : 0u) << (8 * c + e + 1);
          }
      }
      o[f] = word;
    }
    out[idx] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

}  // namespace

extern "C" int mmt_gemm_dropout_keep_bits(const uint32_t* rng, uint32_t layer, uint32_t site, int M,
                                          int N, float keep_prob, int64_t row_offset, uint32_t* out,
                                          mmt_stream_t stream) {
  MMT_CHECK_ARG(rng && out && M > 0 && N > 0 && N % 256 == 0 && keep_prob > 0.f && keep_prob <= 1.f &&
                    (uintptr_t)out % 16 == 0,
                "mmt_gemm_dropout_keep_bits: args (N %% 256 == 0, keep_prob in (0, 1], 16-B aligned out)");
  const int64_t n_words = (int64_t)((M + 255) / 256) * 64 * (N / 32);
  const int blocks = (int)std::min<int64_t>((n_words + 255) / 256, 16384);
  hipLaunchKernelGGL(dropout_keep_words_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), rng, layer,
                     site, keep_threshold16(keep_prob), M, N, row_offset, reinterpret_cast<uint4*>(out),
                     n_words);
  MMT_CHECK_LAUNCH("mmt_gemm_dropout_keep_bits");
  return MMT_OK;
}

extern "C" int mmt_gemm_colsum_rows(int M, int N, int K, int transA, int transB, int c_mode,
                                    int split_k) {
  if (M <= 0 || N <= 0 || K <= 0 || c_mode != MMT_OUT_BF16 || split_k != 1) return 0;
  return nt_bn(M, N, K, transA, transB, 1, 0, 0) == 256 ? (M + 255) / 256 : 0;
}

extern "C" void mmt_gemm_set_variant(int v) { g_variant = v; }

extern "C" int mmt_gemm(int M, int N, int K, const void* A, int transA, int64_t lda,
                        const void* B, int transB, int64_t ldb, void* C, int c_mode, int64_t ldc,
                        int batch, int64_t sA, int64_t sB, int64_t sC, int split_k,
                        const mmt_epilogue_t* e, float* workspace, int64_t ws_elems,
                        mmt_stream_t stream) {
  MMT_CHECK_ARG(A && B && C, "mmt_gemm: null pointer");
  MMT_CHECK_ARG(M > 0 && N > 0 && K > 0 && batch > 0 && split_k > 0, "mmt_gemm: bad shape");
  MMT_CHECK_ARG(c_mode >= MMT_OUT_BF16 && c_mode <= MMT_OUT_F32_ACCUM, "mmt_gemm: c_mode");
  // 16-byte vector loads along the contiguous dimension of each operand; 8-column epilogue
  MMT_CHECK_ARG(((transA ? M : K) % 8 == 0) && lda % 8 == 0 && ((transB ? K : N) % 8 == 0) &&
                    ldb % 8 == 0 && sA % 8 == 0 && sB % 8 == 0 && N % 8 == 0 && ldc % 8 == 0 &&
                    sC % 8 == 0,
                "mmt_gemm: N, contiguous dims and strides must be multiples of 8 (M=%d N=%d K=%d)",
                M, N, K);
  MMT_CHECK_ARG(((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && ((uintptr_t)C % 16 == 0),
                "mmt_gemm: A/B/C not 16-byte aligned");
  MMT_CHECK_ARG(lda >= (transA ? M : K) && ldb >= (transB ? K : N) && ldc >= N,
                "mmt_gemm: leading dimension too small");
  Epi epi{};
  epi.alpha = 1.f;
  if (e) {
    epi.bias = e->bias;
    epi.act = e->act;
    epi.rng = e->rng;
    epi.drop_layer = e->drop_layer;
    epi.drop_site = e->drop_site;
    MMT_CHECK_ARG(!e->rng || (e->keep_prob > 0.f && e->keep_prob <= 1.f), "mmt_gemm: keep_prob");
    epi.keep_thresh16 = e->rng ? keep_threshold16(e->keep_prob) : 65536u;
    epi.drop_scale = e->rng ? 1.f / e->keep_prob : 1.f;
    epi.drop_row_offset = e->drop_row_offset;
    epi.gate = (const bf16_t*)e->gate;
    epi.ld_gate = e->ld_gate;
    epi.gate_scale = e->gate_scale;
    epi.residual = e->residual;
    epi.res_f32 = e->res_dtype == MMT_F32;
    epi.ld_res = e->ld_res;
    epi.alpha = e->alpha;
    epi.beta = e->beta;
    epi.relu_bits = e->relu_bits;
    epi.gate_bits = e->gate_bits;
    MMT_CHECK_ARG(!(e->gate && e->gate_bits), "mmt_gemm: gate and gate_bits are exclusive");
    MMT_CHECK_ARG(!(e->relu_bits && (e->gate_bits || e->colsum)),
                  "mmt_gemm: relu_bits is a forward output (no gate_bits / colsum in that launch)");
    MMT_CHECK_ARG(!e->keep_bits || (e->relu_bits && !e->rng && e->keep_prob > 0.f &&
                                    e->keep_prob <= 1.f && (uintptr_t)e->keep_bits % 16 == 0),
                  "mmt_gemm: keep_bits needs relu_bits, no rng, keep_prob in (0, 1], 16-B alignment");
    epi.keep_bits = e->keep_bits;
    if (e->keep_bits) epi.drop_scale = 1.f / e->keep_prob;
    epi.colsum = e->colsum;
    MMT_CHECK_ARG((!e->gate || (e->ld_gate % 8 == 0 && (uintptr_t)e->gate % 16 == 0)) &&
                      (!e->residual || (e->ld_res % 8 == 0 && (uintptr_t)e->residual % 16 == 0)),
                  "mmt_gemm: gate/residual must be 16-byte aligned with ld % 8 == 0");
    MMT_CHECK_ARG(c_mode != MMT_OUT_F32_ACCUM || (!e->bias && !e->act && !e->rng && !e->gate &&
                                                  !e->residual),
                  "mmt_gemm: accumulate mode takes no epilogue besides alpha");
  }
  hipStream_t s = as_stream(stream);
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int final_kind = c_mode == MMT_OUT_BF16 ? 0 : 1;
  if (c_mode == MMT_OUT_F32_ACCUM) epi.beta = 1.f;  // C += alpha * acc
  int out_kind = final_kind;
  if (split_k > 1) {  // fp32 partial slabs + a combine kernel that applies the epilogue
    MMT_CHECK_ARG(batch == 1, "mmt_gemm: split-K needs batch == 1");
    MMT_CHECK_ARG(workspace && ws_elems >= (int64_t)split_k * M * N &&
                      (uintptr_t)workspace % 16 == 0,
                  "mmt_gemm: split-K needs a 16-B aligned workspace of split_k*M*N floats");
    out_kind = 2;
  }
  // narrow-output NT kernel (products formerly on hipBLASLt)
  if (ntw_ok(M, N, K, transA, transB, batch, out_kind, epi)) {
    const NtwPlan plan = ntw_plan(M, N);
    const int ep = epi.residual ? 1 : epi.act == MMT_ACT_RELU ? 2 : 0;
    auto launch = [&](int mt, int r0, int rows) {
      const int tn = N / plan.bn, n_tiles = ((rows + mt - 1) / mt) * tn;
      int grid = std::min(n_tiles, cu_count());
      if (grid > 8) grid &= ~7;  // XCD-contiguous tile ranges need a multiple of 8 workgroups
      const bf16_t* a = (const bf16_t*)A + (int64_t)r0 * lda;
      bf16_t* c = (bf16_t*)C + (int64_t)r0 * ldc;
      const bf16_t* r = epi.residual ? (const bf16_t*)epi.residual + (int64_t)r0 * epi.ld_res : nullptr;
#define GW(MTV, BNV)                                                                                  \
  do {                                                                                                 \
    if (ep == 0)                                                                                       \
      hipLaunchKernelGGL((gemm_ntw_kernel<MTV, BNV, 0>), dim3(grid), dim3(NTW_NT), 0, s, rows, N, K, a, \
                         lda, (const bf16_t*)B, ldb, c, ldc, r, epi.ld_res, tn, n_tiles);              \
    else if (ep == 1)                                                                                  \
      hipLaunchKernelGGL((gemm_ntw_kernel<MTV, BNV, 1>), dim3(grid), dim3(NTW_NT), 0, s, rows, N, K, a, \
                         lda, (const bf16_t*)B, ldb, c, ldc, r, epi.ld_res, tn, n_tiles);              \
    else                                                                                               \
      hipLaunchKernelGGL((gemm_ntw_kernel<MTV, BNV, 2>), dim3(grid), dim3(NTW_NT), 0, s, rows, N, K, a, \
                         lda, (const bf16_t*)B, ldb, c, ldc, r, epi.ld_res, tn, n_tiles);              \
  } while (0)
      if (plan.bn == 384) {
        switch (mt) {
          case 64: GW(64, 384); break;
          case 128: GW(128, 384); break;
          case 192: GW(192, 384); break;
          default: GW(256, 384); break;
        }
      } else {
        if (mt == 128) GW(128, 192);
        else GW(256, 192);
      }
#undef GW
    };
    if (plan.rows_big > 0) launch(256, 0, plan.rows_big);
    if (M > plan.rows_big) launch(plan.mt2, plan.rows_big, M - plan.rows_big);
    MMT_CHECK_LAUNCH("mmt_gemm(ntw)");
    return MMT_OK;
  }
  // activation-stationary short-K kernel (csrc/gemm_xs.hip) for the bf16 products at K = 384
  // with a bias / relu / dropout / relu-bit epilogue (the OCTO-small QKV projection: 198 vs
  // 220 us at B = 512; the MLP up-projection with relu bits; bit-identical outputs and bit
  // images; tools/xs_bench.py). MMT_XS=0: off (A/B); MMT_XS=1: the bias-only products only.
  if (xs_enabled() && g_variant < 0 && !transA && transB && batch == 1 && out_kind == 0 &&
      final_kind == 0 && M >= 32768 && (epi.act == MMT_ACT_NONE || epi.act == MMT_ACT_RELU) &&
      !epi.gate && !epi.residual && epi.beta == 0.f && !epi.colsum && !epi.gate_bits &&
      !epi.keep_bits && (xs_mode() == 2 || (epi.act == MMT_ACT_NONE && !epi.rng && !epi.relu_bits))) {
    XsEpi xe;
    xe.bias = epi.bias;
    xe.relu = epi.act == MMT_ACT_RELU;
    xe.rng = epi.rng;
    xe.drop_layer = epi.drop_layer;
    xe.drop_site = epi.drop_site;
    xe.keep_thresh16 = epi.keep_thresh16;
    xe.drop_scale = epi.drop_scale;
    xe.drop_row_offset = epi.drop_row_offset;
    xe.alpha = epi.alpha;
    xe.relu_bits = epi.relu_bits;
    if (xs_shape_ok(M, N, K, false, lda, ldb, ldc, A, B, C, xe))
      return xs_launch(M, N, K, false, A, lda, B, ldb, C, ldc, 0, xe, s);
  }
  // Warp-specialised wide NT kernel: bf16 outputs of N % 128 == 0 with the nt256 epilogues that
  // the step uses (bias, relu, dropout, relu_bits, gate_bits, colsum, bf16 / fp32 residual).
  // MMT_NTWS: 0 off, 1 (default) where nt256 would take 192-wide tiles (N % 256 != 0: the QKV
  // projection, 209 vs 247 us at B = 512), 2 everywhere (the 256-wide nt256 tiles measured
  // faster: MLP up 284 vs 299 us, gated dX 252 vs 289; tools/ntws_bench.py)
  const int g_ntws = ntws_mode();
  if (g_ntws && (g_ntws == 2 || N % 256 != 0) && g_variant < 0 && !transA && transB && batch == 1 &&
      out_kind == 0 && final_kind == 0 &&
      K % 64 == 0 && N % 128 == 0 && N >= 1024 && M >= 4096 && !epi.gate && epi.beta == 0.f &&
      (!epi.bias || N <= WS_BIAS) && !(epi.colsum && epi.relu_bits) && !epi.keep_bits) {
    const int tn = N / 128, n_tiles = ((M + 255) / 256) * tn;
    int grid = std::min(n_tiles, cu_count());
    if (grid > 8) grid &= ~7;
#define GWS(CSV, GBV)                                                                                   \
  hipLaunchKernelGGL((gemm_ntws_kernel<CSV, GBV>), dim3(grid), dim3(WS_NT), 0, s, M, N, K,              \
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, (bf16_t*)C, ldc, tn, n_tiles, epi)
    if (epi.colsum && epi.gate_bits) GWS(true, true);
    else if (epi.colsum) GWS(true, false);
    else if (epi.gate_bits) GWS(false, true);
    else GWS(false, false);
#undef GWS
    MMT_CHECK_LAUNCH("mmt_gemm(ntws)");
    return MMT_OK;
  }
  // Persistent 256 x BN NT kernel (variant -1 auto, 5/6/7 force BN 256/192/128)
  const int bn = (epi.bias && N > NT_BIAS_LDS) ? 0
                 : (t5_res768(M, N, epi) && !transA && transB && batch == 1 && out_kind == 0 &&
                    final_kind == 0 && K % 64 == 0 && !epi.bias && epi.act == MMT_ACT_NONE)
                     ? 192
                     : nt_bn(M, N, K, transA, transB, batch, out_kind, final_kind);
  MMT_CHECK_ARG(!(epi.relu_bits || epi.gate_bits) || (bn == 256 && final_kind == 0),
                "mmt_gemm: relu_bits / gate_bits need the 256-wide bf16 nt path (mmt_gemm_colsum_rows)");
  if (bn) {
    static const int g_nt_xcd_order = getenv("MMT_NT_ORDER") ? atoi(getenv("MMT_NT_ORDER")) : 1;
    const int n_cu = cu_count();
    {
      const int tn = N / bn, n_tiles = ((M + 255) / 256) * tn;
      const int grid = std::min(n_tiles, n_cu);
#define GN(BNV, OUT, ST, NSV)                                                                     \
  hipLaunchKernelGGL((gemm_nt256_kernel<BNV, OUT, ST, NSV>), dim3(grid), dim3(NT3), 0, s, M, N, K, \
                     (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, tn, n_tiles, g_nt_xcd_order, epi)
      // the register stash fits 2 waves/SIMD for bf16 at BN <= 192 and fp32 at BN 128;
      // BN 128 has LDS for 3 stages (DMA two K-steps ahead)
      if (epi.gate_bits) {  // 256-wide bf16 (checked above)
        if (epi.colsum)
          hipLaunchKernelGGL((gemm_nt256_kernel<256, 0, NT_SH256, 2, true, true>), dim3(grid), dim3(NT3),
                             0, s, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, tn,
                             n_tiles, g_nt_xcd_order, epi);
        else
          hipLaunchKernelGGL((gemm_nt256_kernel<256, 0, NT_SH256, 2, false, true>), dim3(grid), dim3(NT3),
                             0, s, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, tn,
                             n_tiles, g_nt_xcd_order, epi);
      } else if (epi.colsum) {
        MMT_CHECK_ARG(final_kind == 0 && bn == 256, "mmt_gemm: colsum needs the 256-wide bf16 nt path "
                      "(mmt_gemm_colsum_rows)");
        hipLaunchKernelGGL((gemm_nt256_kernel<256, 0, NT_SH256, 2, true>), dim3(grid), dim3(NT3), 0, s,
                           M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc, tn,
                           n_tiles, g_nt_xcd_order, epi);
      } else if (final_kind == 0) {
        if (bn == 256 && epi.keep_bits)  // relu_bits launch (checked above)
          hipLaunchKernelGGL((gemm_nt256_kernel<256, 0, NT_SH256, 2, false, false, true>), dim3(grid),
                             dim3(NT3), 0, s, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, C, ldc,
                             tn, n_tiles, g_nt_xcd_order, epi);
        else if (bn == 256) GN(256, 0, NT_SH256, 2);
        else if (bn == 192) GN(192, 0, -1, 2);
        else GN(128, 0, -1, 3);
      } else {
        if (bn == 256) GN(256, 1, 0, 2);
        else if (bn == 192) GN(192, 1, 0, 2);
        else GN(128, 1, -1, 3);
      }
#undef GN
      MMT_CHECK_LAUNCH("mmt_gemm(nt256)");
      return MMT_OK;
    }
  }
  MMT_CHECK_ARG(!epi.colsum, "mmt_gemm: colsum needs the 256-wide bf16 nt path (mmt_gemm_colsum_rows)");
  const int k_chunk = ((K + split_k - 1) / split_k + 63) / 64 * 64;
  if (out_kind == 2) split_k = (K + k_chunk - 1) / k_chunk;  // no empty K-splits
  const int n_work = tiles_m * tiles_n * batch * split_k;
  // 0: PIPE 0 / BK 64, 1: PIPE 1 / BK 64, 2: PIPE 1 / BK 128, 3: 256 x 192 tiles
  const int big_work = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2) * batch * split_k;
  // Automatic choice (tools/gemm_bench.py, B = 256 shapes, graph-timed): NT -> direct-to-LDS
  // kernel (equal or better everywhere: +8 % at K = 1536, +22 % on the T5 projections); TN
  // (weight gradients, split-K) -> 256 x 192 tiles when they fill the chip (+12-15 %); otherwise
  // the register-staged 128 x 128 kernel, single stage up to 24 K-steps.
  int pipe;
  if (g_variant >= 0 && g_variant <= 4) pipe = g_variant;
  else if (!transA && transB && K % 8 == 0) pipe = 4;
  else if (transA && !transB && big_work >= 128) pipe = 3;
  else pipe = k_chunk / 64 > 24 ? 0 : 1;
  const int grid_x = n_work;
  void* Cdst = out_kind == 2 ? (void*)workspace : C;
  const int64_t ldd = out_kind == 2 ? (int64_t)N : ldc;
  const int64_t sdd = out_kind == 2 ? (int64_t)M * N : sC;
#define GL1(TA, TB, OUT, P, BKT)                                                                   \
  hipLaunchKernelGGL((gemm_kernel<TA, TB, OUT, P, BKT>), dim3(grid_x), dim3(NTHREADS), 0, s, M, N, \
                     K, (const bf16_t*)A, lda, sA, (const bf16_t*)B, ldb, sB, Cdst, ldd, sdd,     \
                     split_k, k_chunk, tiles_n, n_work, epi)
#define GLB(TA, TB, OUT)                                                                           \
  hipLaunchKernelGGL((gemm_big_kernel<TA, TB, OUT>), dim3(big_work), dim3(NT2), 0, s, M, N, K,     \
                     (const bf16_t*)A, lda, sA, (const bf16_t*)B, ldb, sB, Cdst, ldd, sdd,        \
                     split_k, k_chunk, (N + BN2 - 1) / BN2, big_work, epi)
#define GLG(OUT)                                                                                   \
  hipLaunchKernelGGL((gemm_glds_nt_kernel<OUT>), dim3(grid_x), dim3(NTHREADS), 0, s, M, N, K,      \
                     (const bf16_t*)A, lda, sA, (const bf16_t*)B, ldb, sB, Cdst, ldd, sdd,        \
                     split_k, k_chunk, tiles_n, n_work, epi)
  if (pipe == 4 && !(!transA && transB && K % 8 == 0)) pipe = 1;  // glds path: NT only
  // TN split-K slabs (every weight gradient of the step): the direct-to-LDS TN kernel
  if (pipe == 3 && out_kind == 2 && transA && !transB && batch == 1) {
    const int tn = (N + TN_BN - 1) / TN_BN;
    // 384-row tiles where M divides (every weight gradient of the step: 384 / 1152 / 1536 rows)
    // unless MMT_TN_BM=256; fewer, larger tiles: the split-K factor is the caller's
    static const int g_tn_bm = getenv("MMT_TN_BM") ? atoi(getenv("MMT_TN_BM")) : 384;
    const bool tall = g_tn_bm == 384 && M % 384 == 0 && g_variant != 9;
    const int work = ((M + (tall ? 383 : 255)) / (tall ? 384 : 256)) * tn * split_k;
    // kernel choice (A/B knobs: g_variant 10, 13, 18 via mmt_gemm_set_variant, or MMT_TN_KERNEL):
    //   13 (default) the two-stage kernel on 16x16x32 MFMAs (gemm_tn_dma16_kernel): round 5,
    //      +1.6-3.4 % over 10 at the step's dW shapes (tools/tn_probe.py, interleaved rounds);
    //   10 the two-stage kernel on 32x32x16 (gemm_tn_dma_kernel);
    //   18 the four-stage ring of 32-row K-steps (gemm_tn_r4_kernel; 384-row tiles only): 4-6 %
    //      slower than 13 on K chunks of 4,416 rows, 4 % faster on the out-projection's 1,216-row
    //      chunks (its deeper prologue), so the default takes it for chunks of at most 2,048 rows
    //      (bit-identical slabs).
    // Measured and removed in round 5: a 16-row slice ring, a staggered ping-pong,
    // the ring with its DMA between the MFMA groups, the ring in two barrier-separated phases
    static const int g_tn_kernel = getenv("MMT_TN_KERNEL") ? atoi(getenv("MMT_TN_KERNEL")) : 13;
    const int tnk = (g_variant == 10 || g_variant == 13 || g_variant == 18) ? g_variant : g_tn_kernel;
    if ((tnk == 18 || (tnk == 13 && g_variant < 10 && k_chunk <= 2048)) && tall)
      hipLaunchKernelGGL(gemm_tn_r4_kernel<384>, dim3(work), dim3(TN_NT), 0, s, M, N, K,
                         (const bf16_t*)A, lda, (const bf16_t*)B, ldb, workspace, split_k, k_chunk, tn);
    else if (tnk == 13 && tall)
      hipLaunchKernelGGL(gemm_tn_dma16_kernel<384>, dim3(work), dim3(TN_NT), 0, s, M, N, K,
                         (const bf16_t*)A, lda, (const bf16_t*)B, ldb, workspace, split_k, k_chunk, tn);
    else if (tnk == 13 || tnk == 18)
      hipLaunchKernelGGL(gemm_tn_dma16_kernel<256>, dim3(work), dim3(TN_NT), 0, s, M, N, K,
                         (const bf16_t*)A, lda, (const bf16_t*)B, ldb, workspace, split_k, k_chunk, tn);
    else if (tall)
      hipLaunchKernelGGL(gemm_tn_dma_kernel<384>, dim3(work), dim3(TN_NT), 0, s, M, N, K,
                         (const bf16_t*)A, lda, (const bf16_t*)B, ldb, workspace, split_k, k_chunk, tn);
    else
      hipLaunchKernelGGL(gemm_tn_dma_kernel<256>, dim3(work), dim3(TN_NT), 0, s, M, N, K,
                         (const bf16_t*)A, lda, (const bf16_t*)B, ldb, workspace, split_k, k_chunk, tn);
    MMT_CHECK_LAUNCH("mmt_gemm(tn dma)");
  } else {
#define GL(TA, TB, OUT)                          \
  do {                                           \
    if (pipe == 4) GLG(OUT);                     \
    else if (pipe == 0) GL1(TA, TB, OUT, 0, 64); \
    else if (pipe == 1) GL1(TA, TB, OUT, 1, 64); \
    else if (pipe == 2) GL1(TA, TB, OUT, 1, 128); \
    else GLB(TA, TB, OUT);                       \
  } while (0)
#define GL_OUT(TA, TB)                          \
  do {                                          \
    if (out_kind == 0) GL(TA, TB, 0);           \
    else if (out_kind == 1) GL(TA, TB, 1);      \
    else GL(TA, TB, 2);                         \
  } while (0)
  if (!transA && transB) GL_OUT(false, true);
  else if (!transA && !transB) GL_OUT(false, false);
  else if (transA && !transB) GL_OUT(true, false);
  else GL_OUT(true, true);
  }
#undef GL_OUT
#undef GL
#undef GL1
#undef GLB
#undef GLG
  MMT_CHECK_LAUNCH("mmt_gemm");
  if (out_kind == 2) {
    const int64_t n4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
    if (final_kind == 0)
      hipLaunchKernelGGL(splitk_epilogue_kernel<0>, dim3(blocks), dim3(256), 0, s, workspace,
                         split_k, M, N, C, ldc, epi);
    else
      hipLaunchKernelGGL(splitk_epilogue_kernel<1>, dim3(blocks), dim3(256), 0, s, workspace,
                         split_k, M, N, C, ldc, epi);
    MMT_CHECK_LAUNCH("mmt_gemm(split-K combine)");
  }
  return MMT_OK;
}

extern "C" int mmt_quant_rows_fp8(const void* x, int64_t ld, int rows, int K, void* q, int64_t ldq,
                                  float* scale, mmt_stream_t stream) {
  MMT_CHECK_ARG(x && q && scale && rows > 0 && K > 0 && K % 8 == 0 && ld % 8 == 0 && ldq % 8 == 0 &&
                    (uintptr_t)x % 16 == 0 && (uintptr_t)q % 8 == 0,
                "mmt_quant_rows_fp8: args (K %% 8 == 0, 16-B aligned rows)");
  hipLaunchKernelGGL(quant_rows_fp8_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream),
                     (const bf16_t*)x, ld, rows, K, (uint8_t*)q, ldq, scale);
  MMT_CHECK_LAUNCH("mmt_quant_rows_fp8");
  return MMT_OK;
}

extern "C" int mmt_gemm_fp8(int M, int N, int K, const void* A, int64_t lda, const float* sa,
                            const void* B, int64_t ldb, const float* sb, void* C, int c_mode,
                            int64_t ldc, const mmt_epilogue_t* e, mmt_stream_t stream) {
  MMT_CHECK_ARG(A && B && C && sa && sb && M > 0 && N > 0 && K > 0, "mmt_gemm_fp8: args");
  MMT_CHECK_ARG(K % 64 == 0 && N % 8 == 0 && lda % 16 == 0 && ldb % 16 == 0 && ldc % 8 == 0 &&
                    (uintptr_t)A % 16 == 0 && (uintptr_t)B % 16 == 0 && (uintptr_t)C % 16 == 0 &&
                    (uintptr_t)sb % 16 == 0,
                "mmt_gemm_fp8: K %% 64, N %% 8, 16-B aligned operands / rows / channel scales");
  MMT_CHECK_ARG(c_mode == MMT_OUT_BF16 || c_mode == MMT_OUT_F32, "mmt_gemm_fp8: c_mode");
  Epi epi{};
  epi.alpha = 1.f;
  if (e) {
    epi.bias = e->bias;
    epi.act = e->act;
    epi.rng = e->rng;
    epi.drop_layer = e->drop_layer;
    epi.drop_site = e->drop_site;
    MMT_CHECK_ARG(!e->rng || (e->keep_prob > 0.f && e->keep_prob <= 1.f), "mmt_gemm_fp8: keep_prob");
    epi.keep_thresh16 = e->rng ? keep_threshold16(e->keep_prob) : 65536u;
    epi.drop_scale = e->rng ? 1.f / e->keep_prob : 1.f;
    epi.drop_row_offset = e->drop_row_offset;
    epi.gate = (const bf16_t*)e->gate;
    epi.ld_gate = e->ld_gate;
    epi.gate_scale = e->gate_scale;
    epi.residual = e->residual;
    epi.res_f32 = e->res_dtype == MMT_F32;
    epi.ld_res = e->ld_res;
    epi.alpha = e->alpha;
    epi.beta = e->beta;
    epi.relu_bits = e->relu_bits;
    epi.gate_bits = e->gate_bits;
    MMT_CHECK_ARG(!(e->gate && e->gate_bits), "mmt_gemm: gate and gate_bits are exclusive");
    MMT_CHECK_ARG(!(e->relu_bits && (e->gate_bits || e->colsum)),
                  "mmt_gemm: relu_bits is a forward output (no gate_bits / colsum in that launch)");
    MMT_CHECK_ARG(!e->keep_bits, "mmt_gemm_fp8: keep_bits is a bf16 nt path epilogue (use rng)");
  }
  hipStream_t s = as_stream(stream);
  // K = 768 products with a bf16 output and no gate / residual / beta (the OCTO-base QKV
  // projection and MLP up-projection): the activation-stationary kernel on e4m3 operands
  if (xs_enabled() && g_variant < 0 && c_mode == MMT_OUT_BF16 && M >= 4096 && !epi.gate && !epi.residual &&
      epi.beta == 0.f && !epi.relu_bits && !epi.gate_bits && !(e && e->colsum)) {
    XsEpi xe;
    xe.bias = epi.bias;
    xe.relu = epi.act == MMT_ACT_RELU;
    xe.rng = epi.rng;
    xe.drop_layer = epi.drop_layer;
    xe.drop_site = epi.drop_site;
    xe.keep_thresh16 = epi.keep_thresh16;
    xe.drop_scale = epi.drop_scale;
    xe.drop_row_offset = epi.drop_row_offset;
    xe.alpha = epi.alpha;
    xe.sa = sa;
    xe.sb = sb;
    if (xs_shape_ok(M, N, K, true, lda, ldb, ldc, A, B, C, xe))
      return xs_launch(M, N, K, true, A, lda, B, ldb, C, ldc, 0, xe, s);
  }
  const int tiles_n = (N + F8_BN - 1) / F8_BN, n_work = ((M + F8_BM - 1) / F8_BM) * tiles_n;
  if (c_mode == MMT_OUT_BF16)
    hipLaunchKernelGGL(gemm_fp8_nt_kernel<0>, dim3(n_work), dim3(256), 0, s, M, N, K,
                       (const uint8_t*)A, lda, sa, (const uint8_t*)B, ldb, sb, C, ldc, tiles_n,
                       n_work, epi);
  else
    hipLaunchKernelGGL(gemm_fp8_nt_kernel<1>, dim3(n_work), dim3(256), 0, s, M, N, K,
                       (const uint8_t*)A, lda, sa, (const uint8_t*)B, ldb, sb, C, ldc, tiles_n,
                       n_work, epi);
  MMT_CHECK_LAUNCH("mmt_gemm_fp8");
  return MMT_OK;
}
