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
#else
#define GEMM_TRACE(i) \
  do {                \
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

// tuning knob: 0 = PIPE 0 / BK 64, 1 = PIPE 1 / BK 64, 2 = PIPE 1 / BK 128; other = by K-steps
// per work item (PIPE 1 up to 24 steps of 64)
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
};

// global -> registers for one 128 x 64 (K-contig) or 64 x 128 (MN-contig) operand tile.
// Branch-free: every chunk loads from an address clamped into range (needs the contiguous
// extent to be a multiple of 8, checked by mmt_gemm); store_tile zeroes the out-of-range chunks
// when it writes LDS. Keeping the mask out of the load lets the compiler count vmcnt waits (a
// predicated load forces vmcnt(0)) and leaves the loads in flight until the store.
template <bool KCONTIG, int BKT>
__device__ __forceinline__ void chunk_of(int c, int r0, int k0, int& row, int& kk) {
  if (KCONTIG) {  // [row][k]: BKT/8 chunks of 8 per row
    row = r0 + c / (BKT / 8);
    kk = k0 + (c % (BKT / 8)) * 8;
  } else {        // [k][row]: 16 chunks of 8 per k-row
    kk = k0 + (c >> 4);
    row = r0 + (c & 15) * 8;
  }
}

template <bool KCONTIG, int BKT>
__device__ __forceinline__ void load_tile(const bf16_t* __restrict__ P, int64_t ld, int rows_lim,
                                          int k_lim, int r0, int k0, uint4 (&reg)[Geom<BKT>::Q]) {
#pragma unroll
  for (int q = 0; q < Geom<BKT>::Q; ++q) {
    int row, kk;
    chunk_of<KCONTIG, BKT>(threadIdx.x + q * NTHREADS, r0, k0, row, kk);
    const bf16_t* p = KCONTIG ? P + (int64_t)min(row, rows_lim - 1) * ld + min(kk, k_lim - 8)
                              : P + (int64_t)min(kk, k_lim - 1) * ld + min(row, rows_lim - 8);
    reg[q] = *reinterpret_cast<const uint4*>(p);
  }
}

template <bool KCONTIG, int BKT>
__device__ __forceinline__ void store_tile(bf16_t* __restrict__ S, const uint4 (&reg)[Geom<BKT>::Q],
                                           int rows_lim, int k_lim, int r0, int k0) {
#pragma unroll
  for (int q = 0; q < Geom<BKT>::Q; ++q) {
    const int c = threadIdx.x + q * NTHREADS;
    int row, kk;
    chunk_of<KCONTIG, BKT>(c, r0, k0, row, kk);
    const uint32_t m = (row < rows_lim && kk < k_lim) ? 0xffffffffu : 0u;
    const int off = KCONTIG ? (c / (BKT / 8)) * Geom<BKT>::KCS + (c % (BKT / 8)) * 8
                            : (c >> 4) * MC_STRIDE + (c & 15) * 8;
    *reinterpret_cast<uint4*>(S + off) =
        make_uint4(reg[q].x & m, reg[q].y & m, reg[q].z & m, reg[q].w & m);
  }
}

__device__ __forceinline__ short4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)((__attribute__((address_space(3))) void*)p));
}

// MFMA 32x32x16 operand fragment: lane (r = lane&31, h = lane>>5) holds X[r][k = 8h + j].
template <bool KCONTIG, int KCS>
__device__ __forceinline__ bf16x8 load_frag(const bf16_t* S, int rbase, int ks, int lane) {
  if (KCONTIG) {
    const bf16_t* p = S + (rbase + (lane & 31)) * KCS + ks * 16 + 8 * (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(p);
  } else {
    const int i = lane & 15, q = i >> 2, p4 = i & 3, g = lane >> 4, h = lane >> 5;
    const int col = rbase + 16 * (g & 1) + 4 * p4;
    const int k1 = ks * 16 + 8 * h + q;
    const short4v v1 = tr_read(S + k1 * MC_STRIDE + col);
    const short4v v2 = tr_read(S + (k1 + 4) * MC_STRIDE + col);
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

// XCD-aware bijective remap: blocks b and b+8 share an XCD (round-robin dispatch), so give each
// XCD a contiguous range of tile ids (guide §5.5 T1, bijective form). Speed only.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
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
      for (int a = 0; a < 2; ++a) af[a] = load_frag<A_KC, KCS>(As, wm * 64 + a * 32, ks, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[b] = load_frag<B_KC, KCS>(Bs, wn * 64 + b * 32, ks, lane);
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
    load_tile<A_KC, BK>(A0 + w.bz * sA, lda, M, w.kend, w.m0, k0, ra);
    load_tile<B_KC, BK>(B0 + w.bz * sB, ldb, N, w.kend, w.n0, k0, rb);
  };
  auto store_step = [&](const Work& w, int kt, bf16_t* S) {
    const int k0 = w.kbeg + kt * BK;
    store_tile<A_KC, BK>(S, ra, M, w.kend, w.m0, k0);
    store_tile<B_KC, BK>(S + TILE_ELEMS, rb, N, w.kend, w.n0, k0);
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

// Split-K combine: v = sum_s slab[s][m][n] (fp32), then the GEMM epilogue, 8 columns per thread.
template <int OUT>
__global__ void splitk_epilogue_kernel(const float* __restrict__ ws, int split, int M, int N,
                                       void* __restrict__ Cv, int64_t ldc, Epi epi) {
  const int n8 = N / 8;
  const int64_t total = (int64_t)M * n8;
  const int64_t slab = (int64_t)M * N;
  uint32_t key = 0;
  if (epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int gr = i / n8, gc = (i % n8) * 8;
    const float* p = ws + (int64_t)gr * N + gc;
    float v[8];
    ldw<8>(p, v);
    for (int k = 1; k < split; ++k) {
      float t[8];
      ldw<8>(p + k * slab, t);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += t[e];
    }
    epilogue_w<8>(epi, key, N, gr, gc, v);
    store_w<OUT, 8>(Cv, (int64_t)gr * ldc + gc, epi.beta, v);
  }
}

}  // namespace

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
  const int k_chunk = ((K + split_k - 1) / split_k + 63) / 64 * 64;
  if (out_kind == 2) split_k = (K + k_chunk - 1) / k_chunk;  // no empty K-splits
  const int n_work = tiles_m * tiles_n * batch * split_k;
  // 0: PIPE 0 / BK 64, 1: PIPE 1 / BK 64, 2: PIPE 1 / BK 128
  const int pipe = (g_variant >= 0 && g_variant <= 2) ? g_variant : (k_chunk / 64 > 24 ? 0 : 1);
  const int grid_x = n_work;
  void* Cdst = out_kind == 2 ? (void*)workspace : C;
  const int64_t ldd = out_kind == 2 ? (int64_t)N : ldc;
  const int64_t sdd = out_kind == 2 ? (int64_t)M * N : sC;
#define GL1(TA, TB, OUT, P, BKT)                                                                   \
  hipLaunchKernelGGL((gemm_kernel<TA, TB, OUT, P, BKT>), dim3(grid_x), dim3(NTHREADS), 0, s, M, N, \
                     K, (const bf16_t*)A, lda, sA, (const bf16_t*)B, ldb, sB, Cdst, ldd, sdd,     \
                     split_k, k_chunk, tiles_n, n_work, epi)
#define GL(TA, TB, OUT)                         \
  do {                                          \
    if (pipe == 0) GL1(TA, TB, OUT, 0, 64);     \
    else if (pipe == 1) GL1(TA, TB, OUT, 1, 64); \
    else GL1(TA, TB, OUT, 1, 128);              \
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
#undef GL_OUT
#undef GL
#undef GL1
  MMT_CHECK_LAUNCH("mmt_gemm");
  if (out_kind == 2) {
    const int64_t n8 = (int64_t)M * N / 8;
    const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 4096);
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
