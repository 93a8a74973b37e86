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
// Epilogue: the fp32 accumulator tile is staged through LDS and processed row-major, 8 columns
// per thread, so bias / gate / residual loads and the C store are 16-32 B vector accesses.
// Split-K writes fp32 partial slabs (plain stores) reduced by a second kernel — no atomics.
#include "common.h"

using namespace mmt;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int KC_STRIDE = BK + 8;   // K-contiguous tile [128][72] bf16 (144 B rows)
constexpr int MC_STRIDE = BM + 8;   // M/N-contiguous tile [64][136] bf16 (272 B rows)
constexpr int TILE_ELEMS = 128 * KC_STRIDE;  // >= 64 * MC_STRIDE
constexpr int NTHREADS = 256;
constexpr int CT_STRIDE = BN + 4;   // fp32 epilogue staging tile [128][132]
static_assert(BM * CT_STRIDE * 4 <= 4 * TILE_ELEMS * 2, "epilogue tile must fit the LDS");

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

// global -> registers for one 128 x 64 (K-contig) or 64 x 128 (MN-contig) operand tile
template <bool KCONTIG>
__device__ __forceinline__ void load_tile(const bf16_t* __restrict__ P, int64_t ld, int rows_lim,
                                          int k_lim, int r0, int k0, uint4 (&reg)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = threadIdx.x + q * NTHREADS;
    int row, kk;
    if (KCONTIG) {  // [row][k]: 8 chunks of 8 per row
      row = c >> 3;
      kk = (c & 7) * 8;
      const bool ok = (r0 + row < rows_lim) && (k0 + kk < k_lim);
      reg[q] = ok ? *reinterpret_cast<const uint4*>(P + (int64_t)(r0 + row) * ld + k0 + kk)
                  : make_uint4(0, 0, 0, 0);
    } else {        // [k][row]: 16 chunks of 8 per k-row
      kk = c >> 4;
      row = (c & 15) * 8;
      const bool ok = (k0 + kk < k_lim) && (r0 + row < rows_lim);
      reg[q] = ok ? *reinterpret_cast<const uint4*>(P + (int64_t)(k0 + kk) * ld + r0 + row)
                  : make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile(bf16_t* __restrict__ S, const uint4 (&reg)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = threadIdx.x + q * NTHREADS;
    int off;
    if (KCONTIG) off = (c >> 3) * KC_STRIDE + (c & 7) * 8;
    else off = (c >> 4) * MC_STRIDE + (c & 15) * 8;
    *reinterpret_cast<uint4*>(S + off) = reg[q];
  }
}

__device__ __forceinline__ short4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)((__attribute__((address_space(3))) void*)p));
}

// MFMA 32x32x16 operand fragment: lane (r = lane&31, h = lane>>5) holds X[r][k = 8h + j].
template <bool KCONTIG>
__device__ __forceinline__ bf16x8 load_frag(const bf16_t* S, int rbase, int ks, int lane) {
  if (KCONTIG) {
    const bf16_t* p = S + (rbase + (lane & 31)) * KC_STRIDE + ks * 16 + 8 * (lane >> 5);
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

__device__ __forceinline__ void ld8(const bf16_t* p, float* f) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = __uint_as_float(w[q] << 16);
    f[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// XCD-aware bijective remap: blocks b and b+8 share an XCD (round-robin dispatch), so give each
// XCD a contiguous range of tile ids (guide §5.5 T1, bijective form). Speed only.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <bool TA, bool TB, int OUT>  // OUT: 0 bf16, 1 fp32 (C = epi + beta*C), 2 fp32 split-K slab
__global__ __launch_bounds__(NTHREADS, 2) void gemm_kernel(
    int M, int N, int K, const bf16_t* __restrict__ A, int64_t lda, int64_t sA,
    const bf16_t* __restrict__ B, int64_t ldb, int64_t sB, void* __restrict__ Cv, int64_t ldc,
    int64_t sC, int split_k, int k_chunk, int tiles_n, Epi epi) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE_ELEMS];
  const int bz = blockIdx.z / split_k, ks_id = blockIdx.z - bz * split_k;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = wg / tiles_n, tn = wg - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = ks_id * k_chunk, kend = min(K, kbeg + k_chunk);
  A += bz * sA;
  B += bz * sB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  constexpr bool A_KC = !TA;  // A [M][K]
  constexpr bool B_KC = TB;   // B [N][K]
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[a][b][q] = 0.f;

  uint4 ra[4], rb[4];
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    load_tile<A_KC>(A, lda, M, kend, m0, kbeg, ra);
    load_tile<B_KC>(B, ldb, N, kend, n0, kbeg, rb);
    store_tile<A_KC>(smem, ra);
    store_tile<B_KC>(smem + TILE_ELEMS, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      load_tile<A_KC>(A, lda, M, kend, m0, k0, ra);
      load_tile<B_KC>(B, ldb, N, kend, n0, k0, rb);
    }
    const bf16_t* As = smem + cur * 2 * TILE_ELEMS;
    const bf16_t* Bs = As + TILE_ELEMS;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) af[a] = load_frag<A_KC>(As, wm * 64 + a * 32, ks, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[b] = load_frag<B_KC>(Bs, wn * 64 + b * 32, ks, lane);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    if (more) {
      bf16_t* Ns = smem + (cur ^ 1) * 2 * TILE_ELEMS;
      store_tile<A_KC>(Ns, ra);
      store_tile<B_KC>(Ns + TILE_ELEMS, rb);
    }
    __syncthreads();
  }

  // ---------------- epilogue: stage the fp32 tile through LDS, then 8 columns per thread
  float* Ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int r = wm * 64 + a * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
        Ct[r * CT_STRIDE + wn * 64 + b * 32 + (lane & 31)] = acc[a][b][q];
      }
  __syncthreads();
  uint32_t key = 0;
  if (OUT != 2 && epi.rng) key = stream_key(epi.rng[0], epi.rng[1], epi.drop_layer, epi.drop_site);
  const int c8 = (threadIdx.x & 15) * 8;
  const int gc = n0 + c8;
  if (gc >= N) return;  // N % 8 == 0: whole 8-column groups are in or out
  float bias[8];
  if (OUT != 2 && epi.bias) ld8(epi.bias + gc, bias);
#pragma unroll 2
  for (int r = threadIdx.x >> 4; r < BM; r += NTHREADS / 16) {
    const int gr = m0 + r;
    if (gr >= M) break;
    float v[8];
    {
      const float4 p0 = *reinterpret_cast<const float4*>(Ct + r * CT_STRIDE + c8);
      const float4 p1 = *reinterpret_cast<const float4*>(Ct + r * CT_STRIDE + c8 + 4);
      v[0] = p0.x; v[1] = p0.y; v[2] = p0.z; v[3] = p0.w;
      v[4] = p1.x; v[5] = p1.y; v[6] = p1.z; v[7] = p1.w;
    }
    if (OUT == 2) {  // split-K partial slab
      float* cp = reinterpret_cast<float*>(Cv) + ks_id * sC + (int64_t)gr * ldc + gc;
      *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
      continue;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= epi.alpha;
    if (epi.bias)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias[e];
    if (epi.act == MMT_ACT_RELU)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    if (epi.gate) {
      float g[8];
      ld8(epi.gate + (int64_t)gr * epi.ld_gate + gc, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= (g[e] > 0.f) ? epi.gate_scale : 0.f;
    }
    if (epi.rng) {
      const uint32_t base = (uint32_t)((epi.drop_row_offset + gr) * (int64_t)N + gc);  // even
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const uint32_t d = pair_draw(key, (base + e) >> 1);
        v[e] = ((d & 0xffffu) < epi.keep_thresh16) ? v[e] * epi.drop_scale : 0.f;
        v[e + 1] = ((d >> 16) < epi.keep_thresh16) ? v[e + 1] * epi.drop_scale : 0.f;
      }
    }
    if (epi.residual) {
      float rr[8];
      const int64_t ro = (int64_t)gr * epi.ld_res + gc;
      if (epi.res_f32) ld8(reinterpret_cast<const float*>(epi.residual) + ro, rr);
      else ld8(reinterpret_cast<const bf16_t*>(epi.residual) + ro, rr);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += rr[e];
    }
    if (OUT == 0) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = (uint32_t)f2bf(v[2 * q]) | ((uint32_t)f2bf(v[2 * q + 1]) << 16);
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(Cv) + bz * sC + (int64_t)gr * ldc + gc) =
          make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      float* cp = reinterpret_cast<float*>(Cv) + bz * sC + (int64_t)gr * ldc + gc;
      if (epi.beta != 0.f) {
        float o[8];
        ld8(cp, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += epi.beta * o[e];
      }
      *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// out[m][n] = beta * out[m][n] + alpha * sum_s slab[s][m][n]  (fp32, 4 columns per thread)
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int split, int M, int N,
                                     float* __restrict__ out, int64_t ldo, float alpha, float beta) {
  const int64_t n4 = (int64_t)M * N / 4;
  const int64_t slab = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    const int m = e / N, n = e % N;
    float4 s = *reinterpret_cast<const float4*>(ws + e);
    for (int k = 1; k < split; ++k) {
      const float4 t = *reinterpret_cast<const float4*>(ws + k * slab + e);
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    float4* op = reinterpret_cast<float4*>(out + (int64_t)m * ldo + n);
    const float4 o = beta != 0.f ? *op : make_float4(0, 0, 0, 0);
    *op = make_float4(beta * o.x + alpha * s.x, beta * o.y + alpha * s.y, beta * o.z + alpha * s.z,
                      beta * o.w + alpha * s.w);
  }
}

}  // namespace

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
  int out_kind = c_mode == MMT_OUT_BF16 ? 0 : 1;
  if (c_mode == MMT_OUT_F32_ACCUM) {
    if (split_k == 1) {  // C += alpha * acc directly in the epilogue
      epi.beta = 1.f;
    } else {
      MMT_CHECK_ARG(batch == 1, "mmt_gemm: split-K needs batch == 1");
      MMT_CHECK_ARG(workspace && ws_elems >= (int64_t)split_k * M * N &&
                        (uintptr_t)workspace % 16 == 0,
                    "mmt_gemm: split-K needs a 16-B aligned workspace of split_k*M*N floats");
      out_kind = 2;
    }
  } else {
    MMT_CHECK_ARG(split_k == 1, "mmt_gemm: split_k > 1 needs MMT_OUT_F32_ACCUM");
  }
  int k_chunk = ((K + split_k - 1) / split_k + BK - 1) / BK * BK;
  dim3 grid(tiles_m * tiles_n, 1, batch * split_k);
  void* Cdst = out_kind == 2 ? (void*)workspace : C;
  const int64_t ldd = out_kind == 2 ? (int64_t)N : ldc;
  const int64_t sdd = out_kind == 2 ? (int64_t)M * N : sC;
#define GL(TA, TB, OUT)                                                                            \
  hipLaunchKernelGGL((gemm_kernel<TA, TB, OUT>), grid, dim3(NTHREADS), 0, s, M, N, K,             \
                     (const bf16_t*)A, lda, sA, (const bf16_t*)B, ldb, sB, Cdst, ldd, sdd,        \
                     split_k, k_chunk, tiles_n, epi)
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
  MMT_CHECK_LAUNCH("mmt_gemm");
  if (out_kind == 2) {
    const int64_t n4 = (int64_t)M * N / 4;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, workspace, split_k, M,
                       N, (float*)C, ldc, epi.alpha, 1.f);
    MMT_CHECK_LAUNCH("mmt_gemm(split-K reduce)");
  }
  return MMT_OK;
}
