// Blockwise-causal multi-head attention for gfx950: flash-style forward and backward.
//
// Replaces flax.linen.SelfAttention's dot_product_attention as configured by the reference
// (model_configs/attention_blocks/vanilla_decoder.yaml:19-31; mask from
// tokenizers/token_sequencer.py:313-321 repeated over heads/batch, octo.py:66-68,119):
//   logits = (q / sqrt(Dh)) . k ; where(mask, logits, finfo.min) ; softmax (fp32) ;
//   attention dropout with ONE (L, L) keep-mask broadcast over batch and heads ; . v
// The (B, H, L, L) logits are never materialised. The mask is not a tensor either: it is the
// token-set table of the layer (set ranges + a bitmask of the key sets each query set sees). Per
// 64-wide tile every lane turns it into a 64-bit visibility word (a few range ops per set), so
// masking costs two bit operations per score, and tiles no query of the block sees are skipped;
// waves whose 32 rows lie past L skip the math. T5 mode: an additive fp32 (H, L, L) bias, scale 1.
//
// Layout: qkv rows (b, t) hold [q(H, Dh) | k(H, Dh) | v(H, Dh)] (the fused QKV GEMM output);
// o rows (b, t) hold (H, Dh); lse / delta are (B, H, L) fp32. Dropout keep bits: the two
// word-major images of mmt_dropout_bits (query words for the forward / dQ, key words for dK/dV),
// read as SGPR lane masks (TileMasks).
//
// Forward and dQ: one wave = 32 queries ON THE LANES; S^T = K . Q^T so every score of a query is
// lane-local (registers) and the row max / sum need one cross-half exchange; the S^T accumulator
// is used directly as the B operand of O^T += V^T . P^T (no LDS round trip for P).
// dK/dV: one wave = 32 keys on the lanes; S = Q . K^T and dP = dO . V^T accumulators feed
// dV^T += dO^T . P and dK^T += Q^T . dS directly. V^T, dO^T, Q^T, K^T operands come from
// row-major LDS tiles through ds_read_b64_tr_b16. K/V (resp. Q/dO) tiles are double-buffered in
// LDS and prefetched through registers one tile ahead: one barrier per tile.
#include <math.h>

#include <algorithm>

#include <type_traits>

#include "common.h"

using namespace mmt;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float float2v __attribute__((ext_vector_type(2)));

namespace {

constexpr int MAX_SETS = 16;
constexpr int KT = 64;      // keys (or queries) per LDS tile
constexpr int NT = 256;      // forward threads per workgroup (4 waves x 32 query rows)
constexpr int QB = NT / 2;   // forward query rows per workgroup
// The backward kernels take their workgroup size as a template parameter: 4 waves (128 rows) or
// 2 waves (64 rows), chosen per launch by how well L fills the row blocks (bwd_threads()).
constexpr int MAXL = 4096;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct AttnMask {
  int n_sets;
  int start[MAX_SETS];
  int len[MAX_SETS];
  uint32_t vis[MAX_SETS];  // bit k: query set s sees key set k
  uint32_t causal;         // bit s: inside set s, query q sees key k only if k <= q (Text sets,
                           // token_sequencer.py:76-82: nn.make_causal_mask)
};

__device__ __forceinline__ int set_of(const AttnMask& m, int t) {
  int s = 0;
#pragma unroll 1
  for (int i = 0; i < m.n_sets; ++i)
    if (t >= m.start[i]) s = i;
  return s;
}

// Any visible (query, key) pair for queries [q0, q1) x keys [k0, k1)?  (workgroup-uniform)
__device__ __forceinline__ bool tile_visible(const AttnMask& m, int q0, int q1, int k0, int k1) {
  uint32_t kmask = 0;
  for (int i = 0; i < m.n_sets; ++i)
    if (m.start[i] < k1 && m.start[i] + m.len[i] > k0 && m.len[i] > 0) kmask |= 1u << i;
  for (int i = 0; i < m.n_sets; ++i)
    if (m.start[i] < q1 && m.start[i] + m.len[i] > q0 && m.len[i] > 0 && (m.vis[i] & kmask))
      return true;
  return false;
}

// first key tile >= k0 that queries [q0, q1) see (L if none)
__device__ __forceinline__ int next_key_tile(const AttnMask& m, int q0, int q1, int k0, int L) {
  for (; k0 < L; k0 += KT)
    if (tile_visible(m, q0, q1, k0, min(L, k0 + KT))) return k0;
  return L;
}
__device__ __forceinline__ int next_query_tile(const AttnMask& m, int k0, int k1, int q0, int L) {
  for (; q0 < L; q0 += KT)
    if (tile_visible(m, q0, min(L, q0 + KT), k0, k1)) return q0;
  return L;
}

// Bits [t0, t0 + 64) of the positions covered by the sets selected in `sel`.
__device__ __forceinline__ uint64_t sets_bits(const AttnMask& m, uint32_t sel, int t0) {
  uint64_t r = 0;
  for (int i = 0; i < m.n_sets; ++i) {
    const int a = max(m.start[i] - t0, 0), e = min(m.start[i] + m.len[i] - t0, KT);
    if (((sel >> i) & 1u) && a < e) {
      const uint64_t hi = e >= 64 ? ~0ull : ((1ull << e) - 1ull);
      r |= hi & ~((1ull << a) - 1ull);
    }
  }
  return r;
}

// Bits [a, e) of a 64-bit tile word (0 <= a < e <= 64)
__device__ __forceinline__ uint64_t bit_range(int a, int e) {
  const uint64_t hi = e >= 64 ? ~0ull : ((1ull << e) - 1ull);
  return hi & ~((1ull << a) - 1ull);
}
// Causal set (query-on-lane view): query q of causal set sq does not see the keys of its own set
// after it: clears keys (q, end(sq)) of the tile starting at kt.
__device__ __forceinline__ uint64_t causal_keys(const AttnMask& m, int sq, int q, int kt,
                                                uint64_t vm) {
  if ((m.causal >> sq) & 1u) {
    const int a = max(q + 1 - kt, 0), e = min(m.start[sq] + m.len[sq] - kt, KT);
    if (a < e) vm &= ~bit_range(a, e);
  }
  return vm;
}
// Key-on-lane view: key k of causal set sk is not seen by the queries of its set before it:
// clears queries [start(sk), k) of the tile starting at qt.
__device__ __forceinline__ uint64_t causal_queries(const AttnMask& m, int sk, int k, int qt,
                                                   uint64_t qm) {
  if ((m.causal >> sk) & 1u) {
    const int a = max(m.start[sk] - qt, 0), e = min(k - qt, KT);
    if (a < e) qm &= ~bit_range(a, e);
  }
  return qm;
}

// Bit of accumulator register r of this lane inside a 32-row word pre-shifted by 4*(lane>>5):
// acc row(r) = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
__device__ __forceinline__ constexpr int rbit(int r) { return (r & 3) + 8 * (r >> 2); }
// 2^x as the bare v_exp_f32 (exp2f adds a denormal-range fix-up of four more VALU ops per call;
// arguments here are <= 0 after the max subtraction and results below 2^-126 are negligible)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// all-ones if the bit is set, else 0
__device__ __forceinline__ int bitmask_of(uint32_t w, int b) { return (int)(w << (31 - b)) >> 31; }

__device__ __forceinline__ short4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4v*)((__attribute__((address_space(3))) void*)p));
}

// A-operand fragment of X^T (rows = d) from a row-major LDS tile X[row][d] (stride STR):
// lane (d = dbase + lane&31, h = lane>>5), element j <-> row 16s + 8(j>>2) + 4h + (j&3) (the
// k order of an accumulator used as the next MFMA's operand).
template <int STR>
__device__ __forceinline__ bf16x8 trans_frag(const bf16_t* tile, int row_base, int dbase, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4, h = lane >> 5;
  const int col = dbase + 16 * (g & 1) + 4 * p;
  const int r1 = row_base + 4 * h + q;
  const short4v a = tr_read(tile + r1 * STR + col);
  const short4v b = tr_read(tile + (r1 + 8) * STR + col);
  short8v v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// A/B-operand fragment with the contraction dim contiguous in a row-major LDS tile X[row][d]:
// lane (row = rbase + lane&31, h), element j <-> d = 16s + 8h + j.
template <int STR>
__device__ __forceinline__ bf16x8 row_frag(const bf16_t* tile, int rbase, int s, int lane) {
  return *reinterpret_cast<const bf16x8*>(tile + (rbase + (lane & 31)) * STR + 16 * s +
                                          8 * (lane >> 5));
}

// Same fragment straight from global memory (rows beyond L read as zero). The load itself is
// unconditional (callers clamp rowp to a valid row): a load under a per-lane branch makes the
// compiler drain every outstanding load (vmcnt(0)) at the join, which inside the tile loop would
// also drain the next tile's prefetch.
__device__ __forceinline__ bf16x8 row_frag_global(const bf16_t* rowp, bool valid, int s, int lane) {
  const uint4 v = *reinterpret_cast<const uint4*>(rowp + 16 * s + 8 * (lane >> 5));
  const uint32_t m = valid ? 0xffffffffu : 0u;
  return __builtin_bit_cast(bf16x8, make_uint4(v.x & m, v.y & m, v.z & m, v.w & m));
}

// Dropout keep masks as SGPR lane masks. mmt_dropout_bits stores the square (L, L) keep mask
// twice, word-major with interleaved positions, rows padded to LP = roundup(L, 64) zero words:
//   QF[w][pos(k)]: bit j = keep(32 w + j, k)   (query words: the query-on-lane kernels)
//   KF[w][pos(q)]: bit j = keep(q, 32 w + j)   (key words: the key-on-lane dK/dV kernel)
// pos(8g + 4h + i) = 8g + 2i + h. For a 64-wide tile at t0 (a multiple of 64), the 64-bit pair
// 16u + r of the 64 words X[w][t0 .. t0 + 63] is the lane mask of accumulator register r of the
// 32-wide sub-tile u: element offset 32u + rbit(r) for lanes 0-31 (the 32 lane rows of word w) in
// its low half, offset 32u + rbit(r) + 4 for lanes 32-63 in its high half. So the mask of one
// score is one v_cndmask with its condition read from an SGPR pair (scalar loads of the tile's
// 256 B per wave), instead of a bit extraction per score.
__host__ __device__ __forceinline__ int lp_of(int L) { return (L + 63) & ~63; }
__device__ __forceinline__ int key_of_pos(int p) { return (p & ~7) | ((p & 1) << 2) | ((p >> 1) & 3); }
// v ? keep : 0 with the condition straight from the SGPR pair (one v_cndmask). Written with the
// inverse-ballot builtin, not inline asm: the compiler's hazard recognizer does not look inside
// an asm statement, and a v_cndmask in asm reading a v_exp_f32 result in the next cycle read the
// stale register (gfx950 trans-forwarding hazard: wrong P on some lanes, non-deterministically).
__device__ __forceinline__ float sel_keep(float v, uint64_t m) {
  return __builtin_amdgcn_inverse_ballot_w64(m) ? v : 0.f;
}
// The N lane masks of one (word, tile or 32-wide sub-tile at t0): wave-uniform address, so
// these are scalar loads (indices into m[] must be compile-time constants to stay in SGPRs).
template <int N>
struct TileMasks {
  uint64_t m[N];
  __device__ __forceinline__ void load(const uint32_t* bits, int lp, int w, int t0) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(
        bits + (int64_t)__builtin_amdgcn_readfirstlane(w) * lp + __builtin_amdgcn_readfirstlane(t0));
#pragma unroll
    for (int j = 0; j < N; ++j) m[j] = p[j];
  }
};

typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
// two floats -> one dword of two bf16 (RNE): a single v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  const float2v v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}
// Pack accumulator registers 8s..8s+7 to a bf16 operand fragment (4 v_cvt_pk_bf16_f32).
__device__ __forceinline__ bf16x8 pack_frag(const floatx16& x, int s) {
  const uint4 u = make_uint4(pk2(x[8 * s], x[8 * s + 1]), pk2(x[8 * s + 2], x[8 * s + 3]),
                             pk2(x[8 * s + 4], x[8 * s + 5]), pk2(x[8 * s + 6], x[8 * s + 7]));
  return __builtin_bit_cast(bf16x8, u);
}

// Column sums of output accumulators (rows = head dims d = 32 dsub + rbit(r) + 4 hh, columns =
// the 32 row-lanes of each half-wave), times `scale`, atomically added to gbias[0 .. 32 ND): the
// bias gradient of the fused QKV projection (colsum of dq / dk / dv) without re-reading dqkv.
// Transposed through LDS (`red`: the idle K/V staging buffers, >= waves x 32 ND x 33 floats; rows
// padded to 33 so both phases are bank-conflict free), per-wave sums in `wsum` [waves][32 ND],
// one global atomic per d per workgroup. Every thread of the workgroup must call it.
template <int ND, int NTT>
__device__ __forceinline__ void colsum_atomic(const floatx16 (&acc)[ND], float scale, float* red,
                                              float* wsum, float* gbias, int lane, int wave) {
  constexpr int ROWS = 32 * ND;
  // `red` is the callers' smem[4 * KT * (32 ND + 8)] bf16 staging array: the (NTT / 64) waves'
  // ROWS x 33 fp32 transposes must fit in it for every (Dh, workgroup size) instantiated
  static_assert((NTT / 64) * ROWS * 33 * 4 <= 4 * KT * (32 * ND + 8) * 2,
                "colsum staging exceeds the K/V LDS buffers for this Dh / workgroup size");
  float* rw = red + wave * (ROWS * 33);
  const int hh = lane >> 5, c = lane & 31;
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) rw[(32 * d + rbit(r) + 4 * hh) * 33 + c] = acc[d][r] * scale;
  __syncthreads();
  for (int row = lane; row < ROWS; row += 64) {
    float sum = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) sum += rw[row * 33 + i];
    wsum[wave * ROWS + row] = sum;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ROWS; i += NTT) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < NTT / 64; ++w) sum += wsum[w * ROWS + i];
    grad_add(gbias + i, sum);
  }
  __syncthreads();  // red / wsum may be reused by the next call
}

// Register-staged copy of two KT x DH bf16 tiles (rows r0.., zero past L) -> LDS [KT][DH+8].
// Loads are branch-free (rows clamped to L-1, zeroed at the LDS store), so the compiler keeps
// counted vmcnt waits and the prefetch stays in flight through the MFMAs.
template <int DH, int NTT = NT>
struct TilePair {
  static constexpr int CPR = DH / 8;            // 16-B chunks per row
  static constexpr int PER = KT * CPR / NTT;    // chunks per thread per tile
  uint4 a[PER], b[PER];
  uint32_t ok;
  __device__ __forceinline__ void load(const bf16_t* pa, int64_t sa, const bf16_t* pb, int64_t sb,
                                       int r0, int L) {
    ok = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * NTT, row = c / CPR, ch = c % CPR;
      const int rr = min(r0 + row, L - 1);
      ok |= (r0 + row < L ? 1u : 0u) << i;
      a[i] = *reinterpret_cast<const uint4*>(pa + (int64_t)rr * sa + ch * 8);
      b[i] = *reinterpret_cast<const uint4*>(pb + (int64_t)rr * sb + ch * 8);
    }
  }
  __device__ __forceinline__ void store(bf16_t* la, bf16_t* lb) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * NTT, row = c / CPR, ch = c % CPR;
      const uint32_t m = ((ok >> i) & 1u) ? 0xffffffffu : 0u;
      *reinterpret_cast<uint4*>(la + row * (DH + 8) + ch * 8) =
          make_uint4(a[i].x & m, a[i].y & m, a[i].z & m, a[i].w & m);
      *reinterpret_cast<uint4*>(lb + row * (DH + 8) + ch * 8) =
          make_uint4(b[i].x & m, b[i].y & m, b[i].z & m, b[i].w & m);
    }
  }
};

struct Geo {
  const bf16_t* qkv;
  int64_t s_b, s_t;  // qkv strides (elements)
  int L, H;
  float scale;
};

// A wave's 32 x DH bf16 output rows from O^T-layout accumulators (lane = row r0 + (lane & 31),
// register r of d-subtile d = column 32 d + 8 (r >> 2) + 4 (lane >> 5) + (r & 3)), each row scaled
// by its lane's sc: written to the wave's LDS region `so` (32 x STR, 8 B per lane), read back as
// 16-B row chunks and stored so that every store instruction writes whole 2*DH-byte rows (8 B per
// lane at a row stride would touch 32 rows per instruction). Rows >= L are not stored.
template <int DH, int STR>
__device__ __forceinline__ void store_rows_lds(const floatx16* acc, float sc, bf16_t* so,
                                               bf16_t* base, int64_t row_stride, int r0, int L,
                                               int lane) {
  const int hh = lane >> 5;
#pragma unroll
  for (int d = 0; d < DH / 32; ++d)
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const int dd = 32 * d + 8 * r4 + 4 * hh;
      uint2 w;
      w.x = (uint32_t)f2bf(acc[d][4 * r4] * sc) | ((uint32_t)f2bf(acc[d][4 * r4 + 1] * sc) << 16);
      w.y = (uint32_t)f2bf(acc[d][4 * r4 + 2] * sc) | ((uint32_t)f2bf(acc[d][4 * r4 + 3] * sc) << 16);
      *reinterpret_cast<uint2*>(so + (lane & 31) * STR + dd) = w;
    }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr int CPR = DH / 8;  // 16-B chunks per row
#pragma unroll
  for (int j = 0; j < 32 * CPR / 64; ++j) {
    const int ci = lane + 64 * j, row = ci / CPR, ch = ci - row * CPR;
    if (r0 + row < L)
      *reinterpret_cast<uint4*>(base + (int64_t)(r0 + row) * row_stride + ch * 8) =
          *reinterpret_cast<const uint4*>(so + row * STR + ch * 8);
  }
  __builtin_amdgcn_wave_barrier();  // the region may be rewritten next
}

// =============================================================================== forward
// One workgroup = 4 waves over 128 NQ query rows of one (sample, head): wave w owns the NQ
// 32-row query blocks w, w + 4, ..., each with its own Q fragments, O^T accumulators and
// running max / sum. Every K/V tile is staged into LDS ONCE for all of them: with NQ = 2 one
// workgroup covers L <= 256 rows, so K and V of a (sample, head) are read from HBM once and each
// LDS tile feeds NQ x 16 MFMAs per wave instead of 16, which amortises the per-tile barrier and
// the per-workgroup prologue (the launch picks NQ per L, mmt_attn_fwd).
template <int DH, int NQ, bool WS, bool DROP, int NW = 4>
__global__ __launch_bounds__(64 * NW, DH > 128 ? 1 : 2) void attn_fwd_kernel(
    Geo g, AttnMask mask, const uint32_t* __restrict__ drop_q, int drop_lp, float drop_scale,
    const float* __restrict__ bias, bf16_t* __restrict__ o, int64_t o_s_b, int64_t o_s_t,
    float* __restrict__ lse, float* __restrict__ wsum) {
  constexpr int STR = DH + 8;
  constexpr int NS = DH / 16;   // k-steps over the head dim
  constexpr int ND = DH / 32;   // 32-row d sub-tiles of O^T
  constexpr int TILE = KT * STR;
  // [buf][K | V]; the one-wave form (L <= 32: one key tile) keeps a single buffer, so twice as
  // many of its workgroups fit a CU's LDS (the T5 layers: 6,144 one-wave workgroups)
  constexpr int NBUF = NW == 1 ? 1 : 2;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * NBUF * TILE];
  // visibility word of every (query set, 64-key tile) pair, built once per workgroup
  __shared__ uint64_t s_vis[MAX_SETS * (MAXL / KT)];
  const int b = blockIdx.z, h = blockIdx.y;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = g.L, D = g.H * DH;
  constexpr int NTF = 64 * NW, QBF = 32 * NW;  // threads / query rows per block slot
  const int q0 = blockIdx.x * (QBF * NQ), q1 = min(L, q0 + QBF * NQ);
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  const bf16_t* kbase = base + D + h * DH;
  const bf16_t* vbase = base + 2 * D + h * DH;
  const float c = bias ? 1.f : g.scale * LOG2E;  // score -> log2 units (bias mode converts first)

  bf16x8 qf[NQ][NS];
  floatx16 oacc[NQ][ND];
  float m[NQ], l[NQ], ld[NQ];  // ld: sum of the kept (post-dropout) probabilities, for wsum
  uint32_t visq[NQ];
  int sq[NQ], qrow[NQ];
  bool qv[NQ], live[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int qb = q0 + 32 * (wave + NW * i);
    qrow[i] = qb + (lane & 31);
    qv[i] = qrow[i] < L;
    live[i] = qb < L;  // wave-uniform
    const bf16_t* qp = base + (int64_t)(qv[i] ? qrow[i] : 0) * g.s_t + h * DH;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[i][s] = row_frag_global(qp, qv[i], s, lane);
    sq[i] = qv[i] ? set_of(mask, qrow[i]) : 0;
    visq[i] = qv[i] ? mask.vis[sq[i]] : 0u;
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[i][d][r] = 0.f;
    m[i] = -INFINITY;
    l[i] = 0.f;
    ld[i] = 0.f;
  }

  const int ntiles = (L + KT - 1) / KT;
  for (int e = threadIdx.x; e < mask.n_sets * ntiles; e += NTF) {
    const int st = e / ntiles, t = e - st * ntiles;
    s_vis[st * ntiles + t] = sets_bits(mask, mask.vis[st], t * KT);
  }
  TilePair<DH, NTF> pf;
  int kt = next_key_tile(mask, q0, q1, 0, L);
  if (kt < L) {
    pf.load(kbase, g.s_t, vbase, g.s_t, kt, L);
    pf.store(smem, smem + TILE);
  }
  __syncthreads();
  int buf = 0;
  while (kt < L) {
    const int kn = next_key_tile(mask, q0, q1, kt + KT, L);
    if (kn < L) pf.load(kbase, g.s_t, vbase, g.s_t, kn, L);
    const bf16_t* Ks = smem + buf * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      if (!live[i]) continue;
      uint64_t vm = qv[i] ? s_vis[sq[i] * ntiles + kt / KT] : 0ull;
      if (mask.causal) vm = causal_keys(mask, sq[i], qrow[i], kt, vm);
      if (__all(vm == 0ull)) continue;  // no query of this block sees the tile
      const int q = qrow[i];
      // the tile's second 32-key half lies past L (the T5's L = 32, a last tile of <= 32 keys):
      // skipped whole (its scores would all be masked, its probabilities 0)
      const int nu = kt + 32 < L ? 2 : 1;  // wave-uniform
      floatx16 sacc[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u >= nu) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sacc[u][r] = -INFINITY;
          continue;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) sacc[u][r] = 0.f;
#pragma unroll
        for (int s = 0; s < NS; ++s)
          sacc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Ks, 32 * u, s, lane),
                                                            qf[i][s], sacc[u], 0, 0, 0);
      }
      if (bias) {  // registers 4 r4 .. 4 r4 + 3 hold 4 consecutive keys: one float4 (L % 4 == 0)
        const float* brow = bias + ((int64_t)h * L + (qv[i] ? q : 0)) * L;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            if (u >= nu) continue;
            const int k4 = kt + 32 * u + 8 * r4 + 4 * hh;
            const float4 bv = *reinterpret_cast<const float4*>(brow + min(k4, L - 4));
            const float kb = k4 < L ? LOG2E : 0.f;
            const float bb[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              sacc[u][4 * r4 + e] = sacc[u][4 * r4 + e] * (g.scale * LOG2E) + bb[e] * kb;
          }
      }
      if (!__all(vm == ~0ull)) {  // partially visible tile: masked scores -> -inf
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (u >= nu) continue;
          const uint32_t w = (uint32_t)(vm >> (32 * u)) >> (4 * hh);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mk = bitmask_of(w, rbit(r));
            sacc[u][r] = __int_as_float((__float_as_int(sacc[u][r]) & mk) | (~mk & (int)0xff800000u));
          }
        }
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (u < nu)
#pragma unroll
          for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, sacc[u][r]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m[i], tmax);
      const float mnc = mn == -INFINITY ? 0.f : mn * c;
      const float alpha = fast_exp2(m[i] * c - mnc);  // m = -inf -> 0 (nothing accumulated yet)
      // p = 2^(s c - m) in packed pairs (v_pk_fma / v_pk_add), the row sum before dropout, the
      // dropout keep mask as one v_cndmask per score from the SGPR lane masks
      float2v rs2 = {0.f, 0.f}, rd2 = {0.f, 0.f};
      const float2v cc = {c, c}, mm = {-mnc, -mnc};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u >= nu) continue;
        TileMasks<16> dm;  // dropout lane masks of (query word, key sub-tile): scalar loads
        if constexpr (DROP) dm.load(drop_q, drop_lp, (q0 >> 5) + wave + NW * i, kt + 32 * u);
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          float2v a = {sacc[u][r], sacc[u][r + 1]};
          a = __builtin_elementwise_fma(a, cc, mm);
          float2v pp = {fast_exp2(a.x), fast_exp2(a.y)};
          rs2 += pp;
          if constexpr (DROP) {
            pp.x = sel_keep(pp.x, dm.m[r]);
            pp.y = sel_keep(pp.y, dm.m[r + 1]);
          }
          if (WS) rd2 += pp;
          sacc[u][r] = pp.x;
          sacc[u][r + 1] = pp.y;
        }
      }
      float rs = rs2.x + rs2.y;
      rs += __shfl_xor(rs, 32, 64);
      l[i] = l[i] * alpha + rs;
      if (WS) {  // row sum of the kept probabilities (pruning importance)
        float rd = rd2.x + rd2.y;
        rd += __shfl_xor(rd, 32, 64);
        ld[i] = ld[i] * alpha + rd;
      }
      m[i] = mn;
      if (!__all(alpha == 1.f)) {
#pragma unroll
        for (int d = 0; d < ND; ++d)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[i][d][r] *= alpha;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u >= nu) continue;
        const bf16x8 p0 = pack_frag(sacc[u], 0), p1 = pack_frag(sacc[u], 1);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          oacc[i][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Vs, 32 * u, 32 * d, lane), p0, oacc[i][d], 0, 0, 0);
          oacc[i][d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Vs, 32 * u + 16, 32 * d, lane), p1, oacc[i][d], 0, 0, 0);
        }
      }
    }
    if constexpr (NBUF == 2) {
      if (kn < L) pf.store(smem + (buf ^ 1) * 2 * TILE, smem + (buf ^ 1) * 2 * TILE + TILE);
      __syncthreads();
      buf ^= 1;
    } else {  // single buffer: refill after every wave is done with it (never taken at L <= 64)
      __syncthreads();
      if (kn < L) {
        pf.store(smem, smem + TILE);
        __syncthreads();
      }
    }
    kt = kn;
  }
  // O, scaled and rounded to bf16: with NQ = 2 through LDS (the idle K/V buffers: one 32-row
  // region per wave and query block) as whole-row stores (L = 212: 71.2 -> 67.9 us)
  static_assert(NQ == 1 || NW * NQ * 32 <= 2 * NBUF * KT, "O staging regions must fit the K/V buffers");
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    if (!live[i]) continue;  // wave-uniform
    const float inv = l[i] > 0.f ? drop_scale / l[i] : 0.f;
    if constexpr (NQ == 1) {  // measured faster as direct stores at NQ = 1 (L = 292: 117 vs 137 us)
      if (!qv[i]) continue;
      bf16_t* orow = o + (int64_t)b * o_s_b + (int64_t)qrow[i] * o_s_t + h * DH;
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int dd = 32 * d + 8 * r4 + 4 * hh;
          uint2 w;
          w.x = (uint32_t)f2bf(oacc[i][d][4 * r4] * inv) | ((uint32_t)f2bf(oacc[i][d][4 * r4 + 1] * inv) << 16);
          w.y = (uint32_t)f2bf(oacc[i][d][4 * r4 + 2] * inv) | ((uint32_t)f2bf(oacc[i][d][4 * r4 + 3] * inv) << 16);
          *reinterpret_cast<uint2*>(orow + dd) = w;
        }
    } else {
      store_rows_lds<DH, STR>(oacc[i], inv, smem + (wave * NQ + i) * 32 * STR,
                              o + (int64_t)b * o_s_b + h * DH, o_s_t, q0 + 32 * (wave + NW * i), L,
                              lane);
    }
    if (qv[i] && lane < 32) {
      const int q = qrow[i];
      lse[((int64_t)b * g.H + h) * L + q] = l[i] > 0.f ? m[i] * c * LN2 + logf(l[i]) : -INFINITY;
      if (WS) wsum[((int64_t)b * g.H + h) * L + q] = ld[i] * inv;  // sum_k of the dropped weights
    }
  }
}

// ===================================================== forward, K/V resident in LDS (Dh = 64)
// For the short sequences of the training step (L <= 320: every OCTO-small / tiny layer) the
// whole K and V of one (sample, head) fit in LDS (2 x 40 KB at L = 320), so a workgroup loads
// them ONCE by DMA (global_load_lds, no VGPR staging, no per-tile barrier) and its 4 waves then
// sweep their query blocks with no further synchronisation. Two such workgroups fill the 160 KB
// of a CU. Per 32-row query block a wave makes two passes over the visible key tiles: the exact
// row max (QK^T only), then exp / sum / dropout / pack / P.V, software-pipelined (QK^T of tile
// t + 1 and the K fragments of tile t + 2 are issued ahead of tile t's softmax).
//   LDS image: K rows [0, 32 NTILE) then V rows, 128 B per row, 16-B chunk c of row r stored at
//   chunk c ^ res_sw(r): conflict-free for the K row reads (ds_read_b128, 16 rows per lane group)
//   AND the V transposed reads (ds_read_b64_tr_b16, 4 rows x 64 B per 32-lane half).
//   Rows >= L are copies of row L - 1 (finite; their scores are masked and P = 0 there).
// Query blocks are dealt to the 4 waves by the host (longest-first on the visible-tile counts).
constexpr int RES_TILES = 10;  // 32-key tiles: L <= 320
constexpr int RES_NW = 4;
constexpr int RES_SLOTS = 4;   // query blocks per wave (<= 10 blocks over 4 waves)
constexpr float RES_TAU = 8.f; // one-pass forward: lazy-rescale threshold (log2 units)

struct ResPlan {
  uint32_t tword[MAX_SETS][RES_TILES];  // visible keys [32 t, 32 t + 32) of query set s (bit j)
  uint8_t wblk[RES_NW][RES_SLOTS];      // query blocks of each wave, 0xff-terminated
  uint8_t order[RES_TILES];             // every query block, most visible key tiles first
  int nblk;                             // query blocks: ceil(L / 32)
};

// max / sum of a lane's value and lane l ^ 32's (the two half-waves): one v_permlane32_swap
// (lanes 0-31 of its first result keep their own value, lanes 32-63 get lane l - 32's; the
// second result the other way round), no LDS round trip
__device__ __forceinline__ float halves_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__host__ __device__ __forceinline__ int res_sw(int row) {
  return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
}

// A = X^T fragment [d][row] of a swizzled [row][64] image for rows rbase + 16 ks (+ 8): the
// accumulator-operand k order (transposed reads, conflict-free, see the forward).
__device__ __forceinline__ bf16x8 res_trans(const char* img, int rbase, int dsub, int lane) {
  const int ti = lane & 15, tq = ti >> 2, tp = ti & 3, tg = lane >> 4, hh = lane >> 5;
  const int col = 32 * dsub + 16 * (tg & 1) + 4 * tp;
  const int r1 = rbase + 4 * hh + tq, r2 = r1 + 8;
  const short4v a = tr_read(reinterpret_cast<const bf16_t*>(img + r1 * 128 + 16 * ((col >> 3) ^ res_sw(r1)) + 2 * (col & 7)));
  const short4v b = tr_read(reinterpret_cast<const bf16_t*>(img + r2 * 128 + 16 * ((col >> 3) ^ res_sw(r2)) + 2 * (col & 7)));
  const short8v v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// res_trans split into a per-lane byte offset (o[dsub][read], rows of rbase 0) and the tile base:
// valid for any rbase that is a multiple of 16 (res_sw reads row bits 1-3 only), so a kernel
// keeps four offset registers instead of one address per (tile, half, dsub)
__device__ __forceinline__ void res_trans_offs(int lane, int (&o)[2][2]) {
  const int ti = lane & 15, tq = ti >> 2, tp = ti & 3, tg = lane >> 4, hh = lane >> 5;
#pragma unroll
  for (int dsub = 0; dsub < 2; ++dsub) {
    const int col = 32 * dsub + 16 * (tg & 1) + 4 * tp;
    const int r1 = 4 * hh + tq, r2 = r1 + 8;
    o[dsub][0] = r1 * 128 + 16 * ((col >> 3) ^ res_sw(r1)) + 2 * (col & 7);
    o[dsub][1] = r2 * 128 + 16 * ((col >> 3) ^ res_sw(r2)) + 2 * (col & 7);
  }
}
__device__ __forceinline__ bf16x8 res_trans_at(const char* img_rows, const int (&o)[2]) {
  const short4v a = tr_read(reinterpret_cast<const bf16_t*>(img_rows + o[0]));
  const short4v b = tr_read(reinterpret_cast<const bf16_t*>(img_rows + o[1]));
  const short8v v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int NTILE, bool DROP, bool WS, bool ONEPASS>
__global__ __launch_bounds__(64 * RES_NW, 2) void attn_fwd_res_kernel(
    Geo g, AttnMask mask, ResPlan plan, const uint32_t* __restrict__ drop_q, int drop_lp,
    float drop_scale, bf16_t* __restrict__ o, int64_t o_s_b, int64_t o_s_t, float* __restrict__ lse,
    float* __restrict__ wsum) {
  constexpr int DH = 64, NS = 4, ROWS = 32 * NTILE;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * ROWS * DH];  // [K | V] images
  const int bh = blockIdx.x, b = bh / g.H, h = bh - b * g.H;
  const int lane = threadIdx.x & 63, hh = lane >> 5, lr = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = g.L, D = g.H * DH;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  // ---- DMA K and V into LDS: one wave-instruction = 8 rows x 128 B
  {
    const bf16_t* kb = base + D + h * DH;
    constexpr int PIECES = ROWS / 8;  // per tensor
#if MMT_RES_ABL == 2
    if (L < 0)
#endif
    for (int p = wave; p < 2 * PIECES; p += RES_NW) {
      const int t = p >= PIECES, pr = p - t * PIECES;
      const int row = 8 * pr + (lane >> 3);
      const int c = (lane & 7) ^ res_sw(row);
      const bf16_t* src = kb + t * D + (int64_t)min(row, L - 1) * g.s_t + 8 * c;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(smem + t * ROWS * DH + pr * 512),
                                       16, 0, 0);
    }
  }
  const float c2 = g.scale * LOG2E;
  // per-lane LDS byte offsets of the K row fragments (row lr of a tile, chunk 2s + hh)
  const int swr = res_sw(lr);
  int koff[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = lr * 128 + 16 * ((2 * s + hh) ^ swr);
  // V transposed-read offsets: rows 4 hh + (i >> 2) (+ 8), column 16 (g & 1) + 4 (i & 3) (+ 32 dd)
  const int ti = lane & 15, tq = ti >> 2, tp = ti & 3, tg = lane >> 4;
  const char* smc = reinterpret_cast<const char*>(smem);
  const char* Vimg = smc + ROWS * DH * 2;
  // the first query block's Q fragments, in flight with the DMA
  int slot = 0;
  int blk = plan.wblk[wave][0];
  bf16x8 qf[NS];
  auto load_q = [&](int bk) {
    const int qq = 32 * bk + lr;
    const bool ok = qq < L;
    const bf16_t* qp = base + (int64_t)(ok ? qq : L - 1) * g.s_t + h * DH;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = row_frag_global(qp, ok, s, lane);
  };
  if (blk != 0xff) load_q(blk);
  __syncthreads();  // the DMA landed (vmcnt(0) + barrier)

  // epilogue of a query block: O = acc / l (x 1/keep_prob) as bf16 rows, lse, wsum
  auto finish = [&](const floatx16 (&oacc)[2], const float (&l4)[4], const float (&ld4)[4], float mc,
                    int q, bool qv) {
    float l = (l4[0] + l4[1]) + (l4[2] + l4[3]);
    float ld = (ld4[0] + ld4[1]) + (ld4[2] + ld4[3]);
    l = halves_sum(l);
    if constexpr (WS) ld = halves_sum(ld);
    const float inv = l > 0.f ? drop_scale / l : 0.f;
    bf16_t* orow = o + (int64_t)b * o_s_b + (int64_t)(qv ? q : L - 1) * o_s_t + h * DH;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r4 = 0; r4 < 4; r4 += 2) {
        const uint32_t a0 = pk2(oacc[d][4 * r4] * inv, oacc[d][4 * r4 + 1] * inv);
        const uint32_t a1 = pk2(oacc[d][4 * r4 + 2] * inv, oacc[d][4 * r4 + 3] * inv);
        const uint32_t b0 = pk2(oacc[d][4 * r4 + 4] * inv, oacc[d][4 * r4 + 5] * inv);
        const uint32_t b1 = pk2(oacc[d][4 * r4 + 6] * inv, oacc[d][4 * r4 + 7] * inv);
        const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
#if MMT_RES_ABL == 3
        if (qv && L < 0)
#else
        if (qv)
#endif
          *reinterpret_cast<uint4*>(orow + 32 * d + 8 * r4 + 8 * hh) = make_uint4(x0[0], x1[0], x0[1], x1[1]);
      }
    if (qv && lane < 32) {
      const int64_t ri = ((int64_t)b * g.H + h) * L + q;
      lse[ri] = l > 0.f ? mc * LN2 + logf(l) : -INFINITY;
      if (WS) wsum[ri] = ld * inv;  // sum_k of the dropped weights
    }
  };

  while (blk != 0xff) {  // wave-uniform
    const int q0 = 32 * blk, q = q0 + lr;
    const bool qv = q < L;
    const int qc = qv ? q : L - 1;
    const int sq = set_of(mask, qc);
    const int sq0 = __builtin_amdgcn_readfirstlane(sq);
    // one query set over the block and no causal set: the visibility words are wave-uniform
    const bool uni = mask.causal == 0u && __all(sq == sq0);
    // visibility word of every key tile for this lane's query, fetched ONCE per block (a
    // divergent kernarg read inside the tile loop made the compiler wait vmcnt(0) per tile)
    uint32_t vws[NTILE];
    if (uni) {
#pragma unroll
      for (int t = 0; t < NTILE; ++t) vws[t] = plan.tword[sq0][t];
    } else {
#pragma unroll
      for (int t = 0; t < NTILE; ++t) {
        uint32_t vw = plan.tword[sq][t];
        if ((mask.causal >> sq) & 1u) {  // keys of its own set after q
          const int a0 = max(q + 1 - 32 * t, 0), e0 = min(mask.start[sq] + mask.len[sq] - 32 * t, 32);
          if (a0 < e0) vw &= ~(uint32_t)(bit_range(a0, e0));
        }
        vws[t] = vw;
      }
    }
    // tiles [0, nt): up to the last one any query of the block sees (invisible tiles before it,
    // rare, are computed fully masked)
    int nt = 0;
#pragma unroll
    for (int t = 0; t < NTILE; ++t)
      if (!__all(vws[t] == 0u)) nt = t + 1;
#if MMT_RES_ABL == 1
    nt = 0;
#endif
    const int nblk = slot + 1 < RES_SLOTS ? plan.wblk[wave][slot + 1] : 0xff;
    bf16x8 qn[NS];  // the next block's Q, loaded under this block
    {
      const int bk = nblk != 0xff ? nblk : blk;
      const int qq = 32 * bk + lr;
      const bool ok = qq < L;
      const bf16_t* qp = base + (int64_t)(ok ? qq : L - 1) * g.s_t + h * DH;
#pragma unroll
      for (int s = 0; s < NS; ++s) qn[s] = row_frag_global(qp, ok, s, lane);
    }
    // flash-style online softmax with a deferred rescale, software-pipelined: the QK^T MFMAs of
    // tile t + 1 and the K fragments of tile t + 2 are issued before the softmax of tile t, and
    // tile t's V^T fragments before it, so MFMA / LDS latencies hide under the VALU work
    bf16x8 kr[NS];
    auto kread = [&](int t) {
#pragma unroll
      for (int s = 0; s < NS; ++s) kr[s] = *reinterpret_cast<const bf16x8*>(smc + t * 4096 + koff[s]);
    };
    auto qk = [&]() {
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kr[s], qf[s], acc, 0, 0, 0);
      return acc;
    };
    auto maskw = [&](floatx16& acc, uint32_t vw) {  // partially visible tile: masked scores -> -inf
      if (!__all(vw == 0xffffffffu)) {
        const uint32_t w = vw >> (4 * hh);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int mk = bitmask_of(w, rbit(r));
          acc[r] = __int_as_float((__float_as_int(acc[r]) & mk) | (~mk & (int)0xff800000u));
        }
      }
    };
    // pass 1: the exact row max over the visible keys (QK^T MFMAs and a max per score), so
    // that pass 2's probabilities are exp(s - max) as the softmax defines them: the row's
    // largest weight enters the P.V product as an exact 1.0 (a running max that lags it
    // rounds the dominant weights to bf16: +18 % output error measured)
    // ONEPASS (the default): no such pass — online softmax with a lazy running max (mrun, log2
    // units): a tile rescales the accumulators only when some row's tile max exceeds mrun by
    // more than RES_TAU, so the weights stay <= 2^RES_TAU (exact in fp32; bf16-rounded like every
    // other weight: tests/test_attn_norm_gpu.py test_onepass_forward_within_bf16_tolerance)
    float mrun = -INFINITY;
    if constexpr (!ONEPASS) {
      float mrow = -INFINITY;
      if (nt > 0) kread(0);
#pragma unroll
      for (int t = 0; t < NTILE; ++t) {
        if (t < nt) {  // wave-uniform
          floatx16 S = qk();
          if (t + 1 < NTILE && t + 1 < nt) kread(t + 1);
          maskw(S, vws[t]);
#pragma unroll
          for (int r = 0; r < 16; r += 4) mrow = fmaxf(fmaxf(mrow, fmaxf(S[r], S[r + 1])), fmaxf(S[r + 2], S[r + 3]));
        }
      }
      mrow = halves_max(mrow);
      mrun = mrow == -INFINITY ? -INFINITY : mrow * c2;
    }
    float mc = mrun == -INFINITY ? 0.f : mrun;
    floatx16 oacc[2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[d][r] = 0.f;
    float l4[4] = {0.f, 0.f, 0.f, 0.f}, ld4[4] = {0.f, 0.f, 0.f, 0.f};
    floatx16 Sa;
    // dropout lane masks (scalar loads), one tile ahead: waiting on them at first use stalled
    // every tile
    TileMasks<16> dm[2];
    if constexpr (DROP) dm[0].load(drop_q, drop_lp, blk, 0);
    if (nt > 0) {
      kread(0);
      Sa = qk();
      if (nt > 1) kread(1);
      maskw(Sa, vws[0]);
    }
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      if (t < nt) {  // wave-uniform
        if constexpr (DROP)
          if (t + 1 < NTILE) dm[(t + 1) & 1].load(drop_q, drop_lp, blk, 32 * (t + 1));
        floatx16 Sb;
        if (t + 1 < NTILE && t + 1 < nt) {
          Sb = qk();
          if (t + 2 < NTILE && t + 2 < nt) kread(t + 2);
          maskw(Sb, vws[t + 1]);
        }
        bf16x8 vt[2][2];
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) vt[d][ks] = res_trans(Vimg, 32 * t + 16 * ks, d, lane);
        floatx16 p;
        if constexpr (ONEPASS) {
          // the weights with the running max as it stands, issued before the tile max is known:
          // the exponentials do not wait on its cross-lane reduction and vote; the rare tile that
          // moves a row's max by more than RES_TAU recomputes them (same values as computing them
          // after the test: bit-identical)
#pragma unroll
          for (int r = 0; r < 16; ++r) p[r] = fast_exp2(fmaf(Sa[r], c2, -mc));
          float tm = fmaxf(fmaxf(fmaxf(Sa[0], Sa[1]), fmaxf(Sa[2], Sa[3])), fmaxf(fmaxf(Sa[4], Sa[5]), fmaxf(Sa[6], Sa[7])));
          tm = fmaxf(tm, fmaxf(fmaxf(fmaxf(Sa[8], Sa[9]), fmaxf(Sa[10], Sa[11])), fmaxf(fmaxf(Sa[12], Sa[13]), fmaxf(Sa[14], Sa[15]))));
          tm = halves_max(tm) * c2;
          const bool need = tm > mrun + RES_TAU;  // false for a row with no visible key yet
          if (__any(need)) {  // wave-uniform: rescale only the rows that moved
            const float mnew = need ? tm : mrun;
            // (the accumulators are still 0 while mrun = -inf: alpha 0, never 0 x inf)
            const float alpha = !need ? 1.f : mrun == -INFINITY ? 0.f : fast_exp2(mrun - mnew);
#pragma unroll
            for (int d = 0; d < 2; ++d)
#pragma unroll
              for (int r = 0; r < 16; ++r) oacc[d][r] *= alpha;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              l4[r] *= alpha;
              if constexpr (WS) ld4[r] *= alpha;
            }
            mrun = mnew;
            mc = mrun == -INFINITY ? 0.f : mrun;
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] = fast_exp2(fmaf(Sa[r], c2, -mc));
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) p[r] = fast_exp2(fmaf(Sa[r], c2, -mc));
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float e = p[r];
          l4[r & 3] += e;
          if constexpr (DROP) e = sel_keep(e, dm[t & 1].m[r]);
          if constexpr (WS) ld4[r & 3] += e;
          p[r] = e;
        }
        const bf16x8 p0 = pack_frag(p, 0), p1 = pack_frag(p, 1);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vt[d][0], p0, oacc[d], 0, 0, 0);
          oacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vt[d][1], p1, oacc[d], 0, 0, 0);
        }
        Sa = Sb;
      }
    }
    finish(oacc, l4, ld4, mc, q, qv);
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = qn[s];
    ++slot;
    blk = nblk;
  }
}


// Host plan of the resident forward: per-(query set, key tile) visibility words and the query
// blocks of each wave (longest-processing-time first on the number of visible key tiles).
static bool res_plan(const AttnMask& m, int L, ResPlan& plan) {
  const int nt = (L + 31) / 32;
  if (nt > RES_TILES) return false;
  memset(&plan, 0, sizeof(plan));
  for (int s = 0; s < m.n_sets; ++s)
    for (int t = 0; t < nt; ++t) {
      uint32_t w = 0;
      for (int i = 0; i < m.n_sets; ++i) {
        if (!((m.vis[s] >> i) & 1u) || m.len[i] <= 0) continue;
        const int a = std::max(m.start[i] - 32 * t, 0), e = std::min(m.start[i] + m.len[i] - 32 * t, 32);
        for (int j = a; j < e; ++j) w |= 1u << j;
      }
      plan.tword[s][t] = w;
    }
  memset(plan.wblk, 0xff, sizeof(plan.wblk));
  int cost[RES_TILES], order[RES_TILES];
  for (int i = 0; i < nt; ++i) {
    // key tiles any query of block i sees (its query sets' words; causal sets: all of theirs)
    uint32_t any[RES_TILES] = {0};
    for (int s = 0; s < m.n_sets; ++s)
      if (m.len[s] > 0 && m.start[s] < std::min(L, 32 * i + 32) && m.start[s] + m.len[s] > 32 * i)
        for (int t = 0; t < nt; ++t) any[t] |= plan.tword[s][t];
    cost[i] = 1;  // the block's fixed work (Q load, O store)
    for (int t = 0; t < nt; ++t) cost[i] += any[t] ? 4 : 0;
    order[i] = i;
  }
  std::sort(order, order + nt, [&](int a, int b) { return cost[a] > cost[b] || (cost[a] == cost[b] && a < b); });
  plan.nblk = nt;
  for (int k = 0; k < nt; ++k) plan.order[k] = (uint8_t)order[k];
  int load[RES_NW] = {0}, cnt[RES_NW] = {0};
  for (int k = 0; k < nt; ++k) {
    int best = -1;
    for (int w = 0; w < RES_NW; ++w)
      if (cnt[w] < RES_SLOTS && (best < 0 || load[w] < load[best])) best = w;
    if (best < 0) return false;
    plan.wblk[best][cnt[best]++] = (uint8_t)order[k];
    load[best] += cost[order[k]];
  }
  return true;
}


// (A persistent 8-wave forward with double-buffered K / V, attn_fwd_pers_kernel, measured
// slower than the resident kernel — 185.6 vs 175.3 us at L = 292, B = 512 — and was removed in
// round 5)

// ===================================================== backward, resident operands (Dh = 64)
// One workgroup per (sample, head), two phases over LDS images of the same layout as the
// forward's (res_sw chunk swizzle, rows >= L copies of row L - 1):
//   A (queries on the lanes): K and V resident; per query block S^T = K Q^T, dP^T = V dO^T,
//     P = exp2(S c - lse), dS' = P (keep dP - delta kp), dQ^T += K^T dS'^T (K^T by transposed
//     reads of the K image); the row constants of phase B are written here (rc below);
//   B (keys on the lanes), after a barrier that frees the images: Q and dO resident; per key
//     block S' = Q K^T + rc0, dP' = dO V^T + rc1 (the row constants are the INITIAL accumulators,
//     float4 loads of rc), P = exp2(c S'), dV^T += dO^T P_kept, dK^T += Q^T dS' with
//     dS' = P (keep ? dP' : rc1).
// dS' = dS / (1 / kp): the dropout scale is folded into the dQ / dK / dV store scales.
// rc (the `delta` workspace of mmt_attn_bwd): per (sample, head) two rows of LP = lp_of(L) floats,
//   rc0[q] = -lse[q] / scale (-inf for q >= L: P = 0 on padded rows with no masking) and
//   rc1[q] = -kp rowsum(dO O)[q] (0 for q >= L).
// Query / key blocks are dealt to the 4 waves by the host plan. The fused-QKV bias gradient
// (column sums of dq, dk, dv) is folded per block into 16 partial sums per lane, reduced over
// the lanes and waves through LDS at the end of each phase and added with one atomic per d and
// workgroup.
struct ResPlanB {
  uint32_t qword[MAX_SETS][RES_TILES];  // phase A: keys of tile t that query set s sees
  uint32_t kword[MAX_SETS][RES_TILES];  // phase B: queries of tile t that see key set s
  uint8_t qblk[2 * RES_NW][RES_SLOTS];  // query blocks of each phase-A wave (0xff-terminated)
  uint8_t kblk[2 * RES_NW][RES_SLOTS];  // key blocks of each phase-B wave
  // attn_bwd_res8_kernel's work list (0 items: the static deal above): query blocks (b) and key
  // blocks (0x80 | b) of both phases, longest first
  uint8_t items[2 * RES_TILES];
  int n_items;
};

// DMA of rows [0, 32 NTILE) (clamped to L - 1) of two (row stride s) bf16 tensors into the two
// swizzled images of smem: one wave-instruction = 8 rows x 128 B
template <int ROWS>
__device__ __forceinline__ void res_dma2(bf16_t* smem, const bf16_t* a, int64_t sa, const bf16_t* b,
                                         int64_t sb, int L, int wave, int lane) {
  constexpr int PIECES = ROWS / 8;
#if MMT_RES_ABL == 6
  if (L < 0)
#endif
  for (int p = wave; p < 2 * PIECES; p += RES_NW) {
    const int t = p >= PIECES, pr = p - t * PIECES;
    const int row = 8 * pr + (lane >> 3);
    const int c = (lane & 7) ^ res_sw(row);
    const bf16_t* src = (t ? b : a) + (int64_t)min(row, L - 1) * (t ? sb : sa) + 8 * c;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(smem + t * ROWS * 64 + pr * 512),
                                     16, 0, 0);
  }
}

// Bias-gradient column sums. A block's output accumulators acc[dd][r] (head dim
// d = 32 dd + rbit(r) + 4 hh, one column per lane) are folded into 16 partial sums per lane with
// one v_permlane16_swap + add per pair (acc[0][r], acc[1][r]): lane l of 16-lane row
// rho = (l >> 4) & 3 then holds, for dd = rho & 1, hh = rho >> 1, the sums of acc[dd][r] over
// lanes (l & 15) + 32 hh + {0, 16}.
__device__ __forceinline__ void res_bias_fold(const floatx16 (&acc)[2], float (&b16)[16]) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[0][r]), __float_as_uint(acc[1][r]),
                                                    false, false);
    b16[r] += __uint_as_float(x[0]) + __uint_as_float(x[1]);
  }
}
// End of a phase: the 4 waves' folded sums (times sc) summed through LDS (`red`, 16 KB, free)
// over the 16 lanes of each row; one atomic per d by wave 0. Every thread calls it; it starts and
// ends with a barrier.
__device__ __forceinline__ void res_bias_reduce(const float (&b16)[16], float sc, float* red, float* row,
                                                int wave, int lane) {
  __syncthreads();
  float4* my = reinterpret_cast<float4*>(red + (wave * 64 + lane) * 16);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    my[i] = make_float4(b16[4 * i] * sc, b16[4 * i + 1] * sc, b16[4 * i + 2] * sc, b16[4 * i + 3] * sc);
  __syncthreads();
  if (wave == 0) {
    const int d = lane, hh = (d >> 2) & 1, dd = d >> 5;
    const int r = (d & 3) | (((d & 31) >> 3) << 2), rho = 2 * hh + dd;
    float sum = 0.f;
    for (int w = 0; w < RES_NW; ++w)
#pragma unroll
      for (int j = 0; j < 16; ++j) sum += red[(w * 64 + 16 * rho + j) * 16 + r];
    grad_add(row + d, sum);
  }
  __syncthreads();
}

// store a wave's 32 x 64 rows from O^T-layout accumulators (lane = row), scaled, as bf16 with
// 16-B stores (permlane32 swaps, as the forward's O)
__device__ __forceinline__ void res_store_rows(const floatx16 (&acc)[2], float sc, bf16_t* rowp,
                                               bool valid, int hh) {
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r4 = 0; r4 < 4; r4 += 2) {
      const uint32_t a0 = pk2(acc[d][4 * r4] * sc, acc[d][4 * r4 + 1] * sc);
      const uint32_t a1 = pk2(acc[d][4 * r4 + 2] * sc, acc[d][4 * r4 + 3] * sc);
      const uint32_t b0 = pk2(acc[d][4 * r4 + 4] * sc, acc[d][4 * r4 + 5] * sc);
      const uint32_t b1 = pk2(acc[d][4 * r4 + 6] * sc, acc[d][4 * r4 + 7] * sc);
      const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      if (valid)
        *reinterpret_cast<uint4*>(rowp + 32 * d + 8 * r4 + 8 * hh) = make_uint4(x0[0], x1[0], x0[1], x1[1]);
    }
}

template <int NTILE, bool DROP>
__global__ __launch_bounds__(64 * RES_NW, 2) void attn_bwd_res_kernel(
    Geo g, AttnMask mask, ResPlanB plan, const uint32_t* __restrict__ drop_q,
    const uint32_t* __restrict__ drop_k, int drop_lp, float drop_scale,
    const bf16_t* __restrict__ dout, int64_t d_s_b, int64_t d_s_t, const float* __restrict__ lse,
    const bf16_t* __restrict__ o, int64_t o_s_b, int64_t o_s_t, float* __restrict__ rc,
    bf16_t* __restrict__ dqkv, int64_t dq_s_b, int64_t dq_s_t, float* __restrict__ bias_grad) {
  constexpr int DH = 64, NS = 4, ROWS = 32 * NTILE, LP = ROWS;
  constexpr int IMG_BYTES = 2 * ROWS * DH * 2, RED_BYTES = RES_NW * 64 * 16 * 4;
  __shared__ __attribute__((aligned(16))) char smem_raw[IMG_BYTES > RED_BYTES ? IMG_BYTES : RED_BYTES];
  bf16_t* smem = reinterpret_cast<bf16_t*>(smem_raw);
  const int bh = blockIdx.x, b = bh / g.H, h = bh - b * g.H;
  const int lane = threadIdx.x & 63, hh = lane >> 5, lr = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = g.L, D = g.H * DH;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  const bf16_t* dbase = dout + (int64_t)b * d_s_b + h * DH;
  float* rc0 = rc + (int64_t)bh * 2 * LP;
  float* rc1 = rc0 + LP;
  const float c2 = g.scale * LOG2E;
  const float kp = 1.f / drop_scale;
  const char* img0 = smem_raw;
  const char* img1 = img0 + ROWS * DH * 2;
  int koff[NS];  // row-fragment offsets (row lr of a 32-row tile, chunk 2 s + hh)
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = lr * 128 + 16 * ((2 * s + hh) ^ res_sw(lr));
  float* brow = bias_grad ? bias_grad + h * DH : nullptr;  // += column sums of dq / dk / dv
  const float sc_out = g.scale * drop_scale;                // dQ / dK store scale (dS' = kp dS)

  // ================= phase A: dQ (queries on the lanes), K / V resident
  res_dma2<ROWS>(smem, base + D + h * DH, g.s_t, base + 2 * D + h * DH, g.s_t, L, wave, lane);
  float bq[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) bq[r] = 0.f;
  int slot = 0, blk = plan.qblk[wave][0];
  // the block's Q / dO / O row fragments, loaded under the previous block
  bf16x8 qf[NS], df[NS], of[NS];
  auto load_a = [&](int bk) {
    const int qq = 32 * bk + lr;
    const bool ok = qq < L;
    const int qc_ = ok ? qq : L - 1;
    const bf16_t* qp = base + (int64_t)qc_ * g.s_t + h * DH;
    const bf16_t* dp = dbase + (int64_t)qc_ * d_s_t;
    const bf16_t* op = o + (int64_t)b * o_s_b + (int64_t)qc_ * o_s_t + h * DH;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[s] = row_frag_global(qp, ok, s, lane);
      df[s] = row_frag_global(dp, ok, s, lane);
      of[s] = row_frag_global(op, ok, s, lane);
    }
  };
  if (blk != 0xff) load_a(blk);
  __syncthreads();  // the DMA landed
  while (blk != 0xff) {  // wave-uniform
    const int q = 32 * blk + lr;
    const bool qv = q < L;
    const int qc = qv ? q : L - 1;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) part = fmaf((float)of[s][j], (float)df[s][j], part);
    const float dkp = halves_sum(part) * kp;  // kp delta
    // the next block's operands, in flight under this block (of is free once delta is formed)
    const int nblk = slot + 1 < RES_SLOTS ? plan.qblk[wave][slot + 1] : 0xff;
    bf16x8 qn[NS], dn[NS];
    {
      const int qq = 32 * (nblk != 0xff ? nblk : blk) + lr;
      const bool ok = qq < L;
      const int qc_ = ok ? qq : L - 1;
      const bf16_t* qp = base + (int64_t)qc_ * g.s_t + h * DH;
      const bf16_t* dp = dbase + (int64_t)qc_ * d_s_t;
      const bf16_t* op = o + (int64_t)b * o_s_b + (int64_t)qc_ * o_s_t + h * DH;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        qn[s] = row_frag_global(qp, ok, s, lane);
        dn[s] = row_frag_global(dp, ok, s, lane);
        of[s] = row_frag_global(op, ok, s, lane);
      }
    }
    const float lse2 = qv ? lse[(int64_t)bh * L + q] * LOG2E : INFINITY;
    if (lane < 32) {  // phase B's row constants (padded rows: -inf / 0)
      rc0[q] = qv ? -lse[(int64_t)bh * L + q] / g.scale : -INFINITY;
      rc1[q] = qv ? -dkp : 0.f;
    }
    const int sq = set_of(mask, qc);
    const int sq0 = __builtin_amdgcn_readfirstlane(sq);
    const bool uni = mask.causal == 0u && __all(sq == sq0);
    uint32_t vws[NTILE];
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      uint32_t vw = uni ? plan.qword[sq0][t] : plan.qword[sq][t];
      if (!uni && ((mask.causal >> sq) & 1u)) {
        const int a0 = max(q + 1 - 32 * t, 0), e0 = min(mask.start[sq] + mask.len[sq] - 32 * t, 32);
        if (a0 < e0) vw &= ~(uint32_t)(bit_range(a0, e0));
      }
      vws[t] = vw;
    }
    floatx16 dq[2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[d][r] = 0.f;
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      const uint32_t vw = vws[t];
#if MMT_RES_ABL == 4
      if (L < 0) {
#else
      if (!__all(vw == 0u)) {  // wave-uniform
#endif
        TileMasks<16> dm;
        if constexpr (DROP) dm.load(drop_q, drop_lp, blk, 32 * t);
        floatx16 sacc, pacc;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sacc[r] = 0.f;
          pacc[r] = 0.f;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(img0 + t * 4096 + koff[s]);
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(img1 + t * 4096 + koff[s]);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, df[s], pacc, 0, 0, 0);
        }
        if (!__all(vw == 0xffffffffu)) {  // partially visible tile: masked scores -> -inf
          const uint32_t w = vw >> (4 * hh);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mk = bitmask_of(w, rbit(r));
            sacc[r] = __int_as_float((__float_as_int(sacc[r]) & mk) | (~mk & (int)0xff800000u));
          }
        }
        floatx16 ds;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(fmaf(sacc[r], c2, -lse2));
          float tt = pacc[r];
          if constexpr (DROP) tt = sel_keep(tt, dm.m[r]);
          ds[r] = p * (tt - dkp);
        }
        const bf16x8 d0 = pack_frag(ds, 0), d1 = pack_frag(ds, 1);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dq[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans(img0, 32 * t, d, lane), d0, dq[d], 0, 0, 0);
          dq[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans(img0, 32 * t + 16, d, lane), d1, dq[d], 0, 0, 0);
        }
      }
    }
    res_store_rows(dq, sc_out, dqkv + (int64_t)b * dq_s_b + (int64_t)qc * dq_s_t + h * DH, qv, hh);
    if (brow) res_bias_fold(dq, bq);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[s] = qn[s];
      df[s] = dn[s];
    }
    ++slot;
    blk = nblk;
  }
  // every wave is done with the K / V images, rc is written (the reduce's first barrier)
  if (brow) {
    res_bias_reduce(bq, sc_out, reinterpret_cast<float*>(smem_raw), brow, wave, lane);
  } else {
    __syncthreads();
  }

  // ================= phase B: dK / dV (keys on the lanes), Q / dO resident
  res_dma2<ROWS>(smem, base + h * DH, g.s_t, dbase, d_s_t, L, wave, lane);
  float bk[16], bv[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    bk[r] = 0.f;
    bv[r] = 0.f;
  }
  slot = 0;
  blk = plan.kblk[wave][0];
  bf16x8 kf[NS], vf[NS];  // the key block's K / V row fragments
  auto load_b = [&](int bk_, bf16x8 (&kd)[NS], bf16x8 (&vd)[NS]) {
    const int kk = 32 * bk_ + lr;
    const bool ok = kk < L;
    const bf16_t* kp_ = base + (int64_t)(ok ? kk : L - 1) * g.s_t + D + h * DH;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      kd[s] = row_frag_global(kp_, ok, s, lane);
      vd[s] = row_frag_global(kp_ + D, ok, s, lane);
    }
  };
  if (blk != 0xff) load_b(blk, kf, vf);
  __syncthreads();
  while (blk != 0xff) {
    const int key = 32 * blk + lr;
    const bool kv = key < L;
    const int kc = kv ? key : L - 1;
    const int nblk = slot + 1 < RES_SLOTS ? plan.kblk[wave][slot + 1] : 0xff;
    const int sk = set_of(mask, kc);
    const int sk0 = __builtin_amdgcn_readfirstlane(sk);
    const bool uni = mask.causal == 0u && __all(sk == sk0);
    uint32_t qws[NTILE];
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      uint32_t qw = uni ? plan.kword[sk0][t] : plan.kword[sk][t];
      if (!uni && ((mask.causal >> sk) & 1u)) {  // queries of its own set before the key
        const int a0 = max(mask.start[sk] - 32 * t, 0), e0 = min(key - 32 * t, 32);
        if (a0 < e0) qw &= ~(uint32_t)(bit_range(a0, e0));
      }
      if (!kv) qw = 0u;
      qws[t] = qw;
    }
    floatx16 dk[2], dv[2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dk[d][r] = 0.f;
        dv[d][r] = 0.f;
      }
    // row constants of query rows 32 t + 8 j + 4 hh + {0..3} (the initial accumulators of S'
    // and dP')
    auto load_rc = [&](int t, floatx16& a0, floatx16& a1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 x = *reinterpret_cast<const float4*>(rc0 + 32 * t + 8 * j + 4 * hh);
        const float4 y = *reinterpret_cast<const float4*>(rc1 + 32 * t + 8 * j + 4 * hh);
        a0[4 * j] = x.x; a0[4 * j + 1] = x.y; a0[4 * j + 2] = x.z; a0[4 * j + 3] = x.w;
        a1[4 * j] = y.x; a1[4 * j + 1] = y.y; a1[4 * j + 2] = y.z; a1[4 * j + 3] = y.w;
      }
    };
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      const uint32_t qw = qws[t];
#if MMT_RES_ABL == 5
      if (L < 0) {
#else
      if (!__all(qw == 0u)) {  // wave-uniform
#endif
        TileMasks<16> dm;
        if constexpr (DROP) dm.load(drop_k, drop_lp, blk, 32 * t);
        floatx16 sacc, ca;
        load_rc(t, sacc, ca);
        floatx16 pacc = ca;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8 qr = *reinterpret_cast<const bf16x8*>(img0 + t * 4096 + koff[s]);
          const bf16x8 dr_ = *reinterpret_cast<const bf16x8*>(img1 + t * 4096 + koff[s]);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qr, kf[s], sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dr_, vf[s], pacc, 0, 0, 0);
        }
        if (!__all(qw == 0xffffffffu)) {  // partially visible tile: masked scores -> -inf
          const uint32_t w = qw >> (4 * hh);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mk = bitmask_of(w, rbit(r));
            sacc[r] = __int_as_float((__float_as_int(sacc[r]) & mk) | (~mk & (int)0xff800000u));
          }
        }
        floatx16 pk, ds;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(sacc[r] * c2);
          if constexpr (DROP) {
            const bool keep = __builtin_amdgcn_inverse_ballot_w64(dm.m[r]);
            pk[r] = keep ? p : 0.f;
            ds[r] = p * (keep ? pacc[r] : ca[r]);
          } else {
            pk[r] = p;
            ds[r] = p * pacc[r];
          }
        }
        const bf16x8 p0 = pack_frag(pk, 0), p1 = pack_frag(pk, 1);
        const bf16x8 s0 = pack_frag(ds, 0), s1 = pack_frag(ds, 1);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans(img1, 32 * t, d, lane), p0, dv[d], 0, 0, 0);
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans(img1, 32 * t + 16, d, lane), p1, dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans(img0, 32 * t, d, lane), s0, dk[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans(img0, 32 * t + 16, d, lane), s1, dk[d], 0, 0, 0);
        }
      }
    }
    bf16_t* kro = dqkv + (int64_t)b * dq_s_b + (int64_t)kc * dq_s_t + D + h * DH;
    res_store_rows(dk, sc_out, kro, kv, hh);
    res_store_rows(dv, drop_scale, kro + D, kv, hh);
    if (brow) {
      res_bias_fold(dk, bk);
      res_bias_fold(dv, bv);
    }
    ++slot;
    blk = nblk;
    if (blk != 0xff) load_b(blk, kf, vf);
  }
  if (brow) {
    res_bias_reduce(bk, sc_out, reinterpret_cast<float*>(smem_raw), brow + D, wave, lane);
    res_bias_reduce(bv, drop_scale, reinterpret_cast<float*>(smem_raw), brow + 2 * D, wave, lane);
  }
}

// ============================ backward, all four operands resident, both phases concurrent
// attn_bwd_res_kernel reads K, V, Q and dO twice (a DMA into one phase's images and row
// fragments from HBM in the other: 1.55x the algorithmic bytes at L = 292) and runs its phases
// one after the other, each behind its own DMA; ablations at L = 292, B = 512: 513 us of which
// 110 us are phase-A tiles, 174 us phase-B tiles and ~230 us memory not overlapped with them.
// Here one 8-wave workgroup per (sample, head) holds K, V, Q and dO (4 x 40 KB at L <= 320:
// the CU's 160 KB) loaded once; after a prologue that writes the row constants of every query
// row into LDS (delta = rowsum(dO O) from the dO image and O rows loaded under the DMA, the same
// summation order as the two-phase kernel; round 6: they were a global workspace that phase B
// waited on per key tile, and the images were 32 NTILE rows instead of L rounded to 8), waves 0 .. RES8_NA - 1 run phase A (dQ, queries on the lanes) and the
// rest phase B (dK / dV, keys on the lanes) at the same time, blocks dealt longest-first by
// visible tiles, every row fragment read from the images. Same arithmetic and order per output
// as attn_bwd_res_kernel: bit-identical dQ / dK / dV (the bias column sums add the per-wave
// partials over 3 / 5 waves instead of 4 / 4: equal to summation order).
// Phase-A waves of the 8 (a phase-B key block costs ~1.6x a phase-A query block: 3 + 5 waves
// balance the two phases; the bias sums then run over 3 / 5 waves)
#if MMT_RES_ABL == 9  // diagnostic build (tools/attn_stamps.py): per-wave phase stamps
__device__ unsigned long long g_res8_stamps[8192 * 8 * 6];
#define RES8_STAMP(i)                                                                     \
  do {                                                                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                          \
    if (lane == 0 && blockIdx.x < 8192) g_res8_stamps[(blockIdx.x * 8 + wave) * 6 + (i)] = t_; \
  } while (0)
#else
#define RES8_STAMP(i) \
  do {                \
  } while (0)
#endif
constexpr int RES8_NA = 3;
// Rows per LDS image: L rounded up to 8 (one DMA piece = 8 rows), at most the tile rows. The
// tiles' reads past IR land in the next image (finite rows: masked keys / P = 0 queries there)
// or, after the dO image, in a zeroed slack; the row constants follow.
__host__ __device__ constexpr int res8_rows(int L, int ntile) {
  return ((L + 7) & ~7) < 32 * ntile ? ((L + 7) & ~7) : 32 * ntile;
}
__host__ __device__ constexpr int res8_need(int L, int ntile) {  // + the work-list counter
  return 3 * res8_rows(L, ntile) * 128 + 32 * ntile * 128 + 2 * 32 * ntile * 4 + 16;
}
// static LDS of an instantiation: the largest layout that fits the CU's 160 KB (NTILE 10: L <= 312;
// the host falls back to the two-phase kernel past it), at least the bias partials' 96 KB
__host__ __device__ constexpr int res8_lds(int ntile) {
  return res8_need(32 * ntile, ntile) <= 163840 ? (res8_need(32 * ntile, ntile) > 98304 ? res8_need(32 * ntile, ntile) : 98304)
                                                 : 163840;
}
// DMA of rows [0, 8 np) (clamped to L - 1) of two (row stride s) bf16 tensors into two swizzled
// images at da / db: one wave-instruction = 8 rows x 128 B
__device__ __forceinline__ void res_dma2r(char* da, const bf16_t* a, int64_t sa, char* db, const bf16_t* b,
                                          int64_t sb, int L, int np, int wave, int lane) {
  for (int p = wave; p < 2 * np; p += RES_NW) {
    const int t = p >= np, pr = p - t * np;
    const int row = 8 * pr + (lane >> 3);
    const int c = (lane & 7) ^ res_sw(row);
    const bf16_t* src = (t ? b : a) + (int64_t)min(row, L - 1) * (t ? sb : sa) + 8 * c;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)((t ? db : da) + pr * 1024), 16, 0, 0);
  }
}
template <int NTILE, bool DROP>
__global__ __launch_bounds__(64 * 2 * RES_NW, 1) void attn_bwd_res8_kernel(
    Geo g, AttnMask mask, ResPlanB plan, const uint32_t* __restrict__ drop_q,
    const uint32_t* __restrict__ drop_k, int drop_lp, float drop_scale,
    const bf16_t* __restrict__ dout, int64_t d_s_b, int64_t d_s_t, const float* __restrict__ lse,
    const bf16_t* __restrict__ o, int64_t o_s_b, int64_t o_s_t, float* __restrict__ rc,
    bf16_t* __restrict__ dqkv, int64_t dq_s_b, int64_t dq_s_t, float* __restrict__ bias_grad) {
  constexpr int DH = 64, NS = 4, ROWS = 32 * NTILE, LP = ROWS;
  // K | V | Q | dO images of IR rows each, the zeroed slack, the row constants (res8_lds); the
  // bias partials reuse the space after the phases
  __shared__ __attribute__((aligned(16))) char smem_raw[res8_lds(NTILE)];
  const int bh = blockIdx.x, b = bh / g.H, h = bh - b * g.H;
  const int lane = threadIdx.x & 63, hh = lane >> 5, lr = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = g.L, D = g.H * DH;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  const bf16_t* dbase = dout + (int64_t)b * d_s_b + h * DH;
  const float c2 = g.scale * LOG2E;
  const float kp = 1.f / drop_scale;
  const int IR = res8_rows(L, NTILE), IS = IR * 128;
  const char* imgK = smem_raw;
  const char* imgV = imgK + IS;
  const char* imgQ = imgV + IS;
  const char* imgD = imgQ + IS;
  float* rl0 = reinterpret_cast<float*>(smem_raw + 3 * IS + ROWS * 128);  // rc0 / rc1 (below)
  float* rl1 = rl0 + LP;
  int* wq = reinterpret_cast<int*>(rl1 + LP);  // the work-list counter
  int koff[NS];  // row-fragment offsets (row lr of a 32-row tile, chunk 2 s + hh)
#pragma unroll
  for (int s = 0; s < NS; ++s) koff[s] = lr * 128 + 16 * ((2 * s + hh) ^ res_sw(lr));
  int tro[2][2];  // transposed-read offsets
  res_trans_offs(lane, tro);
  float* brow = bias_grad ? bias_grad + h * DH : nullptr;
  const float sc_out = g.scale * drop_scale;

  RES8_STAMP(0);
  // ---- DMA of the four images (waves 0-3: K and V, waves 4-7: Q and dO), IR rows each; the
  //      O rows and lse of the row constants are loaded under it
  if (wave < RES_NW)
    res_dma2r(smem_raw, base + D + h * DH, g.s_t, smem_raw + IS, base + 2 * D + h * DH, g.s_t, L,
              IR / 8, wave, lane);
  else
    res_dma2r(smem_raw + 2 * IS, base + h * DH, g.s_t, smem_raw + 3 * IS, dbase, d_s_t, L, IR / 8,
              wave - RES_NW, lane);
  {  // the slack after the dO image (read as its rows >= IR): zeros
    const int nsl = (ROWS * 128 - IS) / 16;
    for (int i = threadIdx.x; i < nsl; i += 128 * RES_NW)
      reinterpret_cast<uint4*>(smem_raw + 4 * IS)[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  if (threadIdx.x == 0) *wq = 0;
  const int pq = threadIdx.x;
  const bool pv = pq < ROWS && pq < L;
  bf16x8 orow[8];
  float lq = 0.f;
  if (pv) {
    const bf16_t* op = o + (int64_t)b * o_s_b + (int64_t)pq * o_s_t + h * DH;
#pragma unroll
    for (int c = 0; c < 8; ++c) orow[c] = *reinterpret_cast<const bf16x8*>(op + 8 * c);
    lq = lse[(int64_t)bh * L + pq];
  }
  __syncthreads();  // the DMA landed (vmcnt(0) + barrier)
  RES8_STAMP(1);
  // ---- row constants of every query row: rc0 = -lse / scale (-inf past L), rc1 = -kp delta
  //      (0 past L); delta as the two-phase kernel forms it: chunks 0, 2, 4, 6 and 1, 3, 5, 7
  //      of the row as two fmaf chains, then their sum
  if (pq < ROWS) {
    float v0 = -INFINITY, v1 = 0.f;
    if (pv) {
      float part[2] = {0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const bf16x8 df = *reinterpret_cast<const bf16x8*>(imgD + pq * 128 + 16 * (c ^ res_sw(pq)));
#pragma unroll
        for (int j = 0; j < 8; ++j) part[c & 1] = fmaf((float)orow[c][j], (float)df[j], part[c & 1]);
      }
      v0 = -lq / g.scale;
      v1 = -((part[0] + part[1]) * kp);
    }
    rl0[pq] = v0;
    rl1[pq] = v1;
  }
  __syncthreads();
  RES8_STAMP(2);

  // bias sums: each wave's folded partials through LDS once every wave is done with the images,
  // summed over the 8 waves in wave order (as res_bias_reduce), one atomic per d: dq by wave 0,
  // dk by wave 1, dv by wave 2
  float* red = reinterpret_cast<float*>(smem_raw);  // [3][8 waves][64 lanes][16]
  auto bias_out = [&](const float (&bs)[16], int i, float sc) {
    float4* my = reinterpret_cast<float4*>(red + ((i * 8 + wave) * 64 + lane) * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      my[j] = make_float4(bs[4 * j] * sc, bs[4 * j + 1] * sc, bs[4 * j + 2] * sc, bs[4 * j + 3] * sc);
  };
  auto bias_sum = [&](int i, int w0, int nw, float* dst) {
    const int d = lane, dhh = (d >> 2) & 1, dd = d >> 5;
    const int r = (d & 3) | (((d & 31) >> 3) << 2), rho = 2 * dhh + dd;
    float sum = 0.f;
    for (int w = 0; w < nw; ++w)
#pragma unroll
      for (int j = 0; j < 16; ++j) sum += red[((i * 8 + w0 + w) * 64 + 16 * rho + j) * 16 + r];
    grad_add(dst + d, sum);
  };

  float bq[16], bk[16], bv[16];  // bias-gradient partials (dq, dk, dv column sums)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    bq[r] = 0.f;
    bk[r] = 0.f;
    bv[r] = 0.f;
  }
  // ================= phase A: dQ of query block blk (queries on the lanes)
  auto do_a = [&](int blk) {
    const int q = 32 * blk + lr;
    const bool qv = q < L;
    const int qc = qv ? q : L - 1;
    bf16x8 qf[NS], df[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[s] = *reinterpret_cast<const bf16x8*>(imgQ + blk * 4096 + koff[s]);
      df[s] = *reinterpret_cast<const bf16x8*>(imgD + blk * 4096 + koff[s]);
    }
    const float dkp = -rl1[q];  // kp delta (0 past L)
    const float lse2 = qv ? lse[(int64_t)bh * L + q] * LOG2E : INFINITY;
    const int sq = set_of(mask, qc);
    const int sq0 = __builtin_amdgcn_readfirstlane(sq);
    const bool uni = mask.causal == 0u && __all(sq == sq0);
    uint32_t vws[NTILE];
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      uint32_t vw = uni ? plan.qword[sq0][t] : plan.qword[sq][t];
      if (!uni && ((mask.causal >> sq) & 1u)) {
        const int a0 = max(q + 1 - 32 * t, 0), e0 = min(mask.start[sq] + mask.len[sq] - 32 * t, 32);
        if (a0 < e0) vw &= ~(uint32_t)(bit_range(a0, e0));
      }
      vws[t] = vw;
    }
    floatx16 dq[2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[d][r] = 0.f;
    // the dropout lane masks (scalar loads) one tile ahead: waited for at first use otherwise
    TileMasks<16> dmq[2];
    if constexpr (DROP) dmq[0].load(drop_q, drop_lp, blk, 0);
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      const uint32_t vw = vws[t];
      if constexpr (DROP)
        if (t + 1 < NTILE) dmq[(t + 1) & 1].load(drop_q, drop_lp, blk, 32 * (t + 1));
      if (!__all(vw == 0u)) {  // wave-uniform
        const TileMasks<16>& dm = dmq[t & 1];
        floatx16 sacc, pacc;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sacc[r] = 0.f;
          pacc[r] = 0.f;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(imgK + t * 4096 + koff[s]);
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(imgV + t * 4096 + koff[s]);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, df[s], pacc, 0, 0, 0);
        }
        if (!__all(vw == 0xffffffffu)) {
          const uint32_t w = vw >> (4 * hh);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mk = bitmask_of(w, rbit(r));
            sacc[r] = __int_as_float((__float_as_int(sacc[r]) & mk) | (~mk & (int)0xff800000u));
          }
        }
        floatx16 ds;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(fmaf(sacc[r], c2, -lse2));
          float tt = pacc[r];
          if constexpr (DROP) tt = sel_keep(tt, dm.m[r]);
          ds[r] = p * (tt - dkp);
        }
        const bf16x8 d0 = pack_frag(ds, 0), d1 = pack_frag(ds, 1);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dq[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans_at(imgK + 32 * t * 128, tro[d]), d0, dq[d], 0, 0, 0);
          dq[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans_at(imgK + (32 * t + 16) * 128, tro[d]), d1, dq[d], 0, 0, 0);
        }
      }
    }
    res_store_rows(dq, sc_out, dqkv + (int64_t)b * dq_s_b + (int64_t)qc * dq_s_t + h * DH, qv, hh);
    if (brow) res_bias_fold(dq, bq);
  };
  // ================= phase B: dK / dV of key block blk (keys on the lanes)
  auto do_b = [&](int blk) {
    const int key = 32 * blk + lr;
    const bool kv = key < L;
    const int kc = kv ? key : L - 1;
    bf16x8 kf[NS], vf[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      kf[s] = *reinterpret_cast<const bf16x8*>(imgK + blk * 4096 + koff[s]);
      vf[s] = *reinterpret_cast<const bf16x8*>(imgV + blk * 4096 + koff[s]);
    }
    const int sk = set_of(mask, kc);
    const int sk0 = __builtin_amdgcn_readfirstlane(sk);
    const bool uni = mask.causal == 0u && __all(sk == sk0);
    uint32_t qws[NTILE];
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      uint32_t qw = uni ? plan.kword[sk0][t] : plan.kword[sk][t];
      if (!uni && ((mask.causal >> sk) & 1u)) {
        const int a0 = max(mask.start[sk] - 32 * t, 0), e0 = min(key - 32 * t, 32);
        if (a0 < e0) qw &= ~(uint32_t)(bit_range(a0, e0));
      }
      if (!kv) qw = 0u;
      qws[t] = qw;
    }
    floatx16 dk[2], dv[2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dk[d][r] = 0.f;
        dv[d][r] = 0.f;
      }
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      const uint32_t qw = qws[t];
      if (!__all(qw == 0u)) {  // wave-uniform
        TileMasks<16> dm;
        if constexpr (DROP) dm.load(drop_k, drop_lp, blk, 32 * t);
        floatx16 sacc, ca;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 x = *reinterpret_cast<const float4*>(rl0 + 32 * t + 8 * j + 4 * hh);
          const float4 y = *reinterpret_cast<const float4*>(rl1 + 32 * t + 8 * j + 4 * hh);
          sacc[4 * j] = x.x; sacc[4 * j + 1] = x.y; sacc[4 * j + 2] = x.z; sacc[4 * j + 3] = x.w;
          ca[4 * j] = y.x; ca[4 * j + 1] = y.y; ca[4 * j + 2] = y.z; ca[4 * j + 3] = y.w;
        }
        floatx16 pacc = ca;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8 qr = *reinterpret_cast<const bf16x8*>(imgQ + t * 4096 + koff[s]);
          const bf16x8 dr_ = *reinterpret_cast<const bf16x8*>(imgD + t * 4096 + koff[s]);
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qr, kf[s], sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dr_, vf[s], pacc, 0, 0, 0);
        }
        if (!__all(qw == 0xffffffffu)) {
          const uint32_t w = qw >> (4 * hh);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int mk = bitmask_of(w, rbit(r));
            sacc[r] = __int_as_float((__float_as_int(sacc[r]) & mk) | (~mk & (int)0xff800000u));
          }
        }
        floatx16 pk, ds;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(sacc[r] * c2);
          if constexpr (DROP) {
            const bool keep = __builtin_amdgcn_inverse_ballot_w64(dm.m[r]);
            pk[r] = keep ? p : 0.f;
            ds[r] = p * (keep ? pacc[r] : ca[r]);
          } else {
            pk[r] = p;
            ds[r] = p * pacc[r];
          }
        }
        const bf16x8 p0 = pack_frag(pk, 0), p1 = pack_frag(pk, 1);
        const bf16x8 s0 = pack_frag(ds, 0), s1 = pack_frag(ds, 1);
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans_at(imgD + 32 * t * 128, tro[d]), p0, dv[d], 0, 0, 0);
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans_at(imgD + (32 * t + 16) * 128, tro[d]), p1, dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans_at(imgQ + 32 * t * 128, tro[d]), s0, dk[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(res_trans_at(imgQ + (32 * t + 16) * 128, tro[d]), s1, dk[d], 0, 0, 0);
        }
      }
    }
    bf16_t* kro = dqkv + (int64_t)b * dq_s_b + (int64_t)kc * dq_s_t + D + h * DH;
    res_store_rows(dk, sc_out, kro, kv, hh);
    res_store_rows(dv, drop_scale, kro + D, kv, hh);
    if (brow) {
      res_bias_fold(dk, bk);
      res_bias_fold(dv, bv);
    }
  };
  // the work list (plan.n_items > 0): every block of both phases, longest first (host plan); each
  // wave takes the next item from an LDS counter, so a wave whose SIMD partner runs long takes
  // fewer. Otherwise (deterministic mode: the bias partials per wave must be the same every run)
  // the static deal: query blocks on waves 0 .. RES8_NA - 1, key blocks on the rest.
  const bool dyn = plan.n_items > 0;
  for (int slot = 0;; ++slot) {
    int item;
    if (dyn) {
      int it = 0;
      if (lane == 0) it = atomicAdd(wq, 1);
      it = __builtin_amdgcn_readfirstlane(it);
      if (it >= plan.n_items) break;  // wave-uniform
      item = plan.items[it];
    } else {
      if (slot >= RES_SLOTS) break;
      const int blk = wave < RES8_NA ? plan.qblk[wave][slot] : plan.kblk[wave - RES8_NA][slot];
      if (blk == 0xff) break;  // wave-uniform
      item = wave < RES8_NA ? blk : 0x80 | blk;
    }
    if (item & 0x80) do_b(item & 0x7f);
    else do_a(item);
  }
  RES8_STAMP(3);
  if (brow) {  // over all 8 waves (a wave that took no block of a kind adds exact zeros)
    __syncthreads();
    bias_out(bq, 0, sc_out);
    bias_out(bk, 1, sc_out);
    bias_out(bv, 2, drop_scale);
    __syncthreads();
    if (wave < 3) bias_sum(wave, 0, 2 * RES_NW, brow + wave * D);
  }
  RES8_STAMP(4);
}

// Host plan of the resident backward: the forward's query-side words and query-block deal, and
// the key-side words (queries of tile t that see key set s) and key-block deal.
// Longest-processing-time deal of nt blocks (cost[i]) over nw waves, at most RES_SLOTS each.
static bool res_deal(const int* cost, int nt, int nw, uint8_t (*blk)[RES_SLOTS]) {
  int order[RES_TILES];
  for (int i = 0; i < nt; ++i) order[i] = i;
  std::sort(order, order + nt, [&](int a, int b) { return cost[a] > cost[b] || (cost[a] == cost[b] && a < b); });
  int load[2 * RES_NW] = {0}, cnt[2 * RES_NW] = {0};
  for (int k = 0; k < nt; ++k) {
    int best = -1;
    for (int w = 0; w < nw; ++w)
      if (cnt[w] < RES_SLOTS && (best < 0 || load[w] < load[best])) best = w;
    if (best < 0) return false;
    blk[best][cnt[best]++] = (uint8_t)order[k];
    load[best] += cost[order[k]];
  }
  return true;
}

// Cost of a block: 1 (its fixed work) + 4 per key / query tile any of its rows sees.
static void res_costs(const AttnMask& m, int L, const uint32_t (*word)[RES_TILES], int* cost) {
  const int nt = (L + 31) / 32;
  for (int i = 0; i < nt; ++i) {
    uint32_t any[RES_TILES] = {0};
    for (int s = 0; s < m.n_sets; ++s)
      if (m.len[s] > 0 && m.start[s] < std::min(L, 32 * i + 32) && m.start[s] + m.len[s] > 32 * i)
        for (int t = 0; t < nt; ++t) any[t] |= word[s][t];
    cost[i] = 1;
    for (int t = 0; t < nt; ++t) cost[i] += any[t] ? 4 : 0;
  }
}

// Host plan of the resident backward: the forward's query-side words, the key-side words
// (queries of tile t that see key set s), query blocks dealt over na phase-A waves and key
// blocks over nb phase-B waves (the two-phase kernel: 4 and 4, the forward's query deal).
static bool res_plan_bwd(const AttnMask& m, int L, ResPlanB& pb, int na = RES_NW, int nb = RES_NW) {
  ResPlan pf;
  if (!res_plan(m, L, pf)) return false;
  const int nt = (L + 31) / 32;
  memset(&pb, 0, sizeof(pb));
  memcpy(pb.qword, pf.tword, sizeof(pb.qword));
  memset(pb.qblk, 0xff, sizeof(pb.qblk));
  memset(pb.kblk, 0xff, sizeof(pb.kblk));
  if (na == RES_NW) {
    memcpy(pb.qblk, pf.wblk, sizeof(pf.wblk));
  } else {
    int qc[RES_TILES];
    res_costs(m, L, pb.qword, qc);
    if (!res_deal(qc, nt, na, pb.qblk)) return false;
  }
  for (int s = 0; s < m.n_sets; ++s)
    for (int t = 0; t < nt; ++t) {
      uint32_t w = 0;
      for (int i = 0; i < m.n_sets; ++i) {  // query set i sees key set s
        if (!((m.vis[i] >> s) & 1u) || m.len[i] <= 0) continue;
        const int a = std::max(m.start[i] - 32 * t, 0), e = std::min(m.start[i] + m.len[i] - 32 * t, 32);
        for (int j = a; j < e; ++j) w |= 1u << j;
      }
      pb.kword[s][t] = w;
    }
  int kc[RES_TILES];
  res_costs(m, L, pb.kword, kc);
  return res_deal(kc, nt, nb, pb.kblk);
}

// attn_bwd_res8_kernel's work list: every query block (phase A) and key block (phase B) by
// estimated cost, longest first; a key block costs ~1.6x a query block of the same visible tiles
// (16 MFMAs and two more selects per tile against 12)
static void res8_items(const AttnMask& m, int L, ResPlanB& pb) {
  const int nt = (L + 31) / 32;
  int qc[RES_TILES], kc[RES_TILES], cost[2 * RES_TILES];
  res_costs(m, L, pb.qword, qc);
  res_costs(m, L, pb.kword, kc);
  for (int i = 0; i < nt; ++i) {
    pb.items[i] = (uint8_t)i;
    cost[i] = 5 * qc[i];
    pb.items[nt + i] = (uint8_t)(0x80 | i);
    cost[nt + i] = 8 * kc[i];
  }
  std::stable_sort(pb.items, pb.items + 2 * nt, [&](uint8_t a, uint8_t b) {
    const int ca = cost[(a & 0x80) ? nt + (a & 0x7f) : a], cb = cost[(b & 0x80) ? nt + (b & 0x7f) : b];
    return ca > cb;
  });
  pb.n_items = 2 * nt;
}

// =============================================================================== bwd: dQ
template <int DH, int NTT, bool DROP>
__global__ __launch_bounds__(NTT, DH > 128 ? 1 : 2) void attn_bwd_dq_kernel(Geo g, AttnMask mask,
                                                         const uint32_t* __restrict__ drop_q,
                                                         int drop_lp, float drop_scale,
                                                         const bf16_t* __restrict__ dout,
                                                         int64_t d_s_b, int64_t d_s_t,
                                                         const float* __restrict__ lse,
                                                         const bf16_t* __restrict__ o,
                                                         int64_t o_s_b, int64_t o_s_t,
                                                         float* __restrict__ delta,
                                                         bf16_t* __restrict__ dqkv,
                                                         int64_t dq_s_b, int64_t dq_s_t,
                                                         float* __restrict__ bgrad) {
  constexpr int STR = DH + 8;
  constexpr int NS = DH / 16;
  constexpr int ND = DH / 32;
  constexpr int TILE = KT * STR;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE];  // [buf][K | V]
  __shared__ float s_wsum[NTT / 64 * DH];
  // 1-D grid of (sample, head, query block) items, XCD-contiguous: the query blocks of one
  // (sample, head) share an XCD, so its K/V tiles are fetched into one L2 once
  const int nqb = (g.L + NTT / 2 - 1) / (NTT / 2);
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = item / nqb, b = bh / g.H, h = bh - b * g.H;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = g.L, D = g.H * DH;
  const int q0 = (item - bh * nqb) * (NTT / 2), q1 = min(L, q0 + NTT / 2);
  const int q = q0 + wave * 32 + (lane & 31);
  const bool qv = q < L;
  const bool wave_live = q0 + wave * 32 < L;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  const bf16_t* kbase = base + D + h * DH;
  const bf16_t* vbase = base + 2 * D + h * DH;
  bf16x8 qf[NS], df[NS];
  const bf16_t* qrow = base + (int64_t)(qv ? q : 0) * g.s_t + h * DH;
  const bf16_t* drow = dout + (int64_t)b * d_s_b + (int64_t)(qv ? q : 0) * d_s_t + h * DH;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    qf[s] = row_frag_global(qrow, qv, s, lane);
    df[s] = row_frag_global(drow, qv, s, lane);
  }
  const int sq = qv ? set_of(mask, q) : 0;
  const uint32_t visq = qv ? mask.vis[sq] : 0u;
  const int64_t row_bh = ((int64_t)b * g.H + h) * L;
  const float lse2 = qv ? lse[row_bh + q] * LOG2E : INFINITY;
  // delta = rowsum(dO * O) of this query (fp32), fused here: the lane pair (q, hh = 0/1) holds
  // dO[d = 16 s + 8 h + j]; the dK/dV kernel, launched next on the stream, reads it back.
  float dlt;
  {
    const bf16_t* orow = o + (int64_t)b * o_s_b + (int64_t)(qv ? q : 0) * o_s_t + h * DH;
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 of = row_frag_global(orow, qv, s, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) part = fmaf((float)of[j], (float)df[s][j], part);
    }
    dlt = part + __shfl_xor(part, 32, 64);
    if (qv && lane < 32) delta[row_bh + q] = dlt;
  }
  const float sl2 = g.scale * LOG2E;
  floatx16 dqacc[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dqacc[d][r] = 0.f;

  TilePair<DH, NTT> pf;
  int kt = next_key_tile(mask, q0, q1, 0, L);
  if (kt < L) {
    pf.load(kbase, g.s_t, vbase, g.s_t, kt, L);
    pf.store(smem, smem + TILE);
  }
  __syncthreads();
  int buf = 0;
  while (kt < L) {
    const int kn = next_key_tile(mask, q0, q1, kt + KT, L);
    if (kn < L) pf.load(kbase, g.s_t, vbase, g.s_t, kn, L);
    const bf16_t* Ks = smem + buf * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
    if (wave_live) {
      uint64_t vm = sets_bits(mask, visq, kt);
      if (mask.causal) vm = causal_keys(mask, sq, q, kt, vm);
      const bool full = __all(vm == ~0ull);  // wave-uniform: no visibility masking needed
      floatx16 ds[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        TileMasks<16> dm;  // dropout lane masks of (query word, key sub-tile): scalar loads
        if constexpr (DROP) dm.load(drop_q, drop_lp, (q0 >> 5) + wave, kt + 32 * u);
        floatx16 sacc, pacc;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sacc[r] = 0.f;
          pacc[r] = 0.f;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Ks, 32 * u, s, lane), qf[s],
                                                         sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Vs, 32 * u, s, lane), df[s],
                                                         pacc, 0, 0, 0);
        }
        const uint32_t wv = (uint32_t)(vm >> (32 * u)) >> (4 * hh);
        const float2v sl = {sl2, sl2}, ml = {-lse2, -lse2}, dd = {drop_scale, drop_scale},
                      dl = {dlt, dlt};
        // one wave-uniform branch between the fully visible form and the masked one (a per-pair
        // branch would be emitted around every inline-asm select otherwise)
        auto scores = [&](auto full_t) {
          constexpr bool FULL = decltype(full_t)::value;
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            float2v a = {sacc[r], sacc[r + 1]};
            a = __builtin_elementwise_fma(a, sl, ml);
            float2v pp = {fast_exp2(a.x), fast_exp2(a.y)};
            if constexpr (!FULL) {
              pp.x = __int_as_float(__float_as_int(pp.x) & bitmask_of(wv, rbit(r)));
              pp.y = __int_as_float(__float_as_int(pp.y) & bitmask_of(wv, rbit(r + 1)));
            }
            float2v t = {pacc[r], pacc[r + 1]};
            t *= dd;
            if constexpr (DROP) {
              t.x = sel_keep(t.x, dm.m[r]);
              t.y = sel_keep(t.y, dm.m[r + 1]);
            }
            const float2v dsp = pp * (t - dl);
            ds[u][r] = dsp.x;
            ds[u][r + 1] = dsp.y;
          }
        };
        if (full) scores(std::true_type{});
        else scores(std::false_type{});
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const bf16x8 p0 = pack_frag(ds[u], 0), p1 = pack_frag(ds[u], 1);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          dqacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Ks, 32 * u, 32 * d, lane), p0, dqacc[d], 0, 0, 0);
          dqacc[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Ks, 32 * u + 16, 32 * d, lane), p1, dqacc[d], 0, 0, 0);
        }
      }
    }
    if (kn < L) pf.store(smem + (buf ^ 1) * 2 * TILE, smem + (buf ^ 1) * 2 * TILE + TILE);
    __syncthreads();
    buf ^= 1;
    kt = kn;
  }
  if (bgrad)  // kernel-uniform; the loop's last barrier freed the staging buffers
    colsum_atomic<ND, NTT>(dqacc, g.scale, reinterpret_cast<float*>(smem), s_wsum,
                           bgrad + h * DH, lane, wave);
  // the loop's last barrier (or colsum_atomic's) freed the staging buffers
  store_rows_lds<DH, STR>(dqacc, g.scale, smem + wave * 32 * STR, dqkv + (int64_t)b * dq_s_b + h * DH,
                          dq_s_t, q - (lane & 31), L, lane);
}

// =============================================================================== bwd: dK, dV
template <int DH, int NTT, bool DROP>
__global__ __launch_bounds__(NTT, DH > 128 ? 1 : 2) void attn_bwd_dkdv_kernel(Geo g, AttnMask mask,
                                                           const uint32_t* __restrict__ drop_k,
                                                           int drop_lp, float drop_scale,
                                                           const bf16_t* __restrict__ dout,
                                                           int64_t d_s_b, int64_t d_s_t,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           bf16_t* __restrict__ dqkv,
                                                           int64_t dq_s_b, int64_t dq_s_t,
                                                           float* __restrict__ bgrad) {
  constexpr int STR = DH + 8;
  constexpr int NS = DH / 16;
  constexpr int ND = DH / 32;
  constexpr int TILE = KT * STR;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE];  // [buf][Q | dO]
  __shared__ __attribute__((aligned(16))) float s_rows[2][2][KT];  // [buf][lse*log2e | delta]
  __shared__ float s_wsum[NTT / 64 * DH];
  // 1-D grid of (sample, head, key block) items, XCD-contiguous: the key blocks of one
  // (sample, head) share an XCD, so its Q/dO tiles are fetched into one L2 once
  const int nkb = (g.L + NTT / 2 - 1) / (NTT / 2);
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = item / nkb, b = bh / g.H, h = bh - b * g.H;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int L = g.L, D = g.H * DH;
  const int kb0 = (item - bh * nkb) * (NTT / 2), kb1 = min(L, kb0 + NTT / 2);
  const int key = kb0 + wave * 32 + (lane & 31);
  const bool kv = key < L;
  const bool wave_live = kb0 + wave * 32 < L;
  const bf16_t* base = g.qkv + (int64_t)b * g.s_b;
  const bf16_t* qbase = base + h * DH;
  const bf16_t* dbase = dout + (int64_t)b * d_s_b + h * DH;
  bf16x8 kf[NS], vf[NS];
  const bf16_t* krow = base + (int64_t)(kv ? key : 0) * g.s_t + D + h * DH;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = row_frag_global(krow, kv, s, lane);
    vf[s] = row_frag_global(krow + D, kv, s, lane);
  }
  // query sets that see this key's set
  uint32_t selq = 0;
  const int sk = kv ? set_of(mask, key) : 0;
  if (kv)
    for (int i = 0; i < mask.n_sets; ++i) selq |= ((mask.vis[i] >> sk) & 1u) << i;
  const int64_t row_bh = ((int64_t)b * g.H + h) * L;
  const float sl2 = g.scale * LOG2E;
  floatx16 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dk[d][r] = 0.f;
      dv[d][r] = 0.f;
    }

  TilePair<DH, NTT> pf;
  float rowv = 0.f;  // thread t < 128 stages lse (t < 64) or delta (64 <= t < 128) of one row
  auto load_rows = [&](int q0) {  // waves 0 (lse) and 1 (delta); clamped, branch-free load
    if (threadIdx.x < 2 * KT) {
      const int qq = q0 + (threadIdx.x & (KT - 1));
      const float v = (threadIdx.x < KT ? lse : delta)[row_bh + min(qq, L - 1)];
      rowv = threadIdx.x < KT ? (qq < L ? v * LOG2E : INFINITY) : (qq < L ? v : 0.f);
    }
  };
  auto store_rows = [&](int bi) {
    if (threadIdx.x < 2 * KT) s_rows[bi][threadIdx.x >> 6][threadIdx.x & (KT - 1)] = rowv;
  };
  int qt = next_query_tile(mask, kb0, kb1, 0, L);
  if (qt < L) {
    pf.load(qbase, g.s_t, dbase, d_s_t, qt, L);
    load_rows(qt);
    pf.store(smem, smem + TILE);
    store_rows(0);
  }
  __syncthreads();
  int buf = 0;
  while (qt < L) {
    const int qn = next_query_tile(mask, kb0, kb1, qt + KT, L);
    if (qn < L) {
      pf.load(qbase, g.s_t, dbase, d_s_t, qn, L);
      load_rows(qn);
    }
    const bf16_t* Qs = smem + buf * 2 * TILE;
    const bf16_t* Ds = Qs + TILE;
    if (wave_live) {
      uint64_t qm = sets_bits(mask, selq, qt);
      if (mask.causal) qm = causal_queries(mask, sk, key, qt, qm);
      const bool full = __all(qm == ~0ull);  // wave-uniform: no visibility masking needed
#pragma unroll 1
      for (int u = 0; u < 2; ++u) {  // 32-query sub-tiles (not unrolled: keeps 2 waves/SIMD)
        TileMasks<16> dm;  // dropout lane masks of (key word, query sub-tile): scalar loads
        if constexpr (DROP) dm.load(drop_k, drop_lp, (kb0 >> 5) + wave, qt + 32 * u);
        floatx16 sacc, pacc;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sacc[r] = 0.f;
          pacc[r] = 0.f;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Qs, 32 * u, s, lane), kf[s],
                                                         sacc, 0, 0, 0);
          pacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(row_frag<STR>(Ds, 32 * u, s, lane), vf[s],
                                                         pacc, 0, 0, 0);
        }
        // per-row lse / delta: rows 32u + 8j + 4hh + {0..3} are float4 j
        float lr[16], dr[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 a = *reinterpret_cast<const float4*>(&s_rows[buf][0][32 * u + 8 * j + 4 * hh]);
          const float4 d = *reinterpret_cast<const float4*>(&s_rows[buf][1][32 * u + 8 * j + 4 * hh]);
          lr[4 * j] = a.x; lr[4 * j + 1] = a.y; lr[4 * j + 2] = a.z; lr[4 * j + 3] = a.w;
          dr[4 * j] = d.x; dr[4 * j + 1] = d.y; dr[4 * j + 2] = d.z; dr[4 * j + 3] = d.w;
        }
        const uint32_t wv = (uint32_t)(qm >> (32 * u)) >> (4 * hh);
        floatx16 pd, dsv;
        const float2v sl = {sl2, sl2}, dd = {drop_scale, drop_scale};
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          float2v a = {sacc[r], sacc[r + 1]};
          const float2v ml = {-lr[r], -lr[r + 1]}, dl = {dr[r], dr[r + 1]};
          a = __builtin_elementwise_fma(a, sl, ml);
          float2v pp = {fast_exp2(a.x), fast_exp2(a.y)};
          if (!full) {
            pp.x = __int_as_float(__float_as_int(pp.x) & bitmask_of(wv, rbit(r)));
            pp.y = __int_as_float(__float_as_int(pp.y) & bitmask_of(wv, rbit(r + 1)));
          }
          float2v t = {pacc[r], pacc[r + 1]};
          t *= dd;
          float2v pk = pp;  // drop_scale applied to dV at the end
          if constexpr (DROP) {
            pk.x = sel_keep(pp.x, dm.m[r]);
            pk.y = sel_keep(pp.y, dm.m[r + 1]);
            t.x = sel_keep(t.x, dm.m[r]);
            t.y = sel_keep(t.y, dm.m[r + 1]);
          }
          const float2v dsp = pp * (t - dl);
          pd[r] = pk.x;
          pd[r + 1] = pk.y;
          dsv[r] = dsp.x;
          dsv[r + 1] = dsp.y;
        }
        const bf16x8 pd0 = pack_frag(pd, 0), pd1 = pack_frag(pd, 1);
        const bf16x8 ds0 = pack_frag(dsv, 0), ds1 = pack_frag(dsv, 1);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trans_frag<STR>(Ds, 32 * u, 32 * d, lane),
                                                          pd0, dv[d], 0, 0, 0);
          dv[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Ds, 32 * u + 16, 32 * d, lane), pd1, dv[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trans_frag<STR>(Qs, 32 * u, 32 * d, lane),
                                                          ds0, dk[d], 0, 0, 0);
          dk[d] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              trans_frag<STR>(Qs, 32 * u + 16, 32 * d, lane), ds1, dk[d], 0, 0, 0);
        }
      }
    }
    if (qn < L) {
      pf.store(smem + (buf ^ 1) * 2 * TILE, smem + (buf ^ 1) * 2 * TILE + TILE);
      store_rows(buf ^ 1);
    }
    __syncthreads();
    buf ^= 1;
    qt = qn;
  }
  if (bgrad) {  // kernel-uniform: bias gradients of the K and V projections
    colsum_atomic<ND, NTT>(dk, g.scale, reinterpret_cast<float*>(smem), s_wsum,
                           bgrad + D + h * DH, lane, wave);
    colsum_atomic<ND, NTT>(dv, drop_scale, reinterpret_cast<float*>(smem), s_wsum,
                           bgrad + 2 * D + h * DH, lane, wave);
  }
  bf16_t* kbase_o = dqkv + (int64_t)b * dq_s_b + D + h * DH;
  store_rows_lds<DH, STR>(dk, g.scale, smem + wave * 32 * STR, kbase_o, dq_s_t, key - (lane & 31),
                          L, lane);
  store_rows_lds<DH, STR>(dv, drop_scale, smem + wave * 32 * STR, kbase_o + D, dq_s_t,
                          key - (lane & 31), L, lane);
}

// =============================================================================== dropout bits
// Non-square masks (out_t == null): row-major words (rows, W), bit j of word (r, w) = keep(r,
// 32 w + j). Square attention masks: the two word-major interleaved images QF (out) and KF
// (out_t) described at TileMasks, W x LP words each, zero past L.
__global__ void dropout_bits_kernel(const uint32_t* __restrict__ rng, uint32_t layer, uint32_t site,
                                    int rows, int cols, int words, uint32_t thresh,
                                    uint32_t* __restrict__ out, uint32_t* __restrict__ out_t) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t key = stream_key(rng[0], rng[1], layer, site);
  uint32_t bits = 0;
  if (!out_t) {
    if (idx >= (int64_t)rows * words) return;
    const int r = idx / words, w = idx % words;
    for (int j = 0; j < 32; ++j) {
      const int c = w * 32 + j;
      if (c < cols && keep_elem(key, (uint32_t)((int64_t)r * cols + c), thresh)) bits |= 1u << j;
    }
    out[idx] = bits;
    return;
  }
  const int L = rows, lp = lp_of(L);
  const int64_t n = (int64_t)words * lp;
  if (idx >= 2 * n) return;
  const bool kimg = idx >= n;
  const int64_t t = kimg ? idx - n : idx;
  const int w = t / lp, x = key_of_pos((int)(t % lp));
  if (x < L)
    for (int j = 0; j < 32; ++j) {
      const int y = w * 32 + j;  // QF: row y, column x; KF: row x, column y
      const int r = kimg ? x : y, c = kimg ? y : x;
      if (y < L && keep_elem(key, (uint32_t)((int64_t)r * cols + c), thresh)) bits |= 1u << j;
    }
  (kimg ? out_t : out)[t] = bits;
}

int fill_mask(AttnMask& m, int n_sets, const int32_t* starts, const int32_t* lens,
              const uint32_t* vis, int L) {
  m.causal = 0;
  if (n_sets <= 0) {  // no mask: one set covering everything
    m.n_sets = 1;
    m.start[0] = 0;
    m.len[0] = L;
    m.vis[0] = 1u;
    for (int i = 1; i < MAX_SETS; ++i) {
      m.start[i] = 1 << 30;
      m.len[i] = 0;
      m.vis[i] = 0;
    }
    return MMT_OK;
  }
  MMT_CHECK_ARG(n_sets <= MAX_SETS && starts && lens && vis, "attention: bad token-set table");
  m.n_sets = n_sets;
  int expect = 0;
  for (int i = 0; i < n_sets; ++i) {
    MMT_CHECK_ARG(starts[i] == expect && lens[i] >= 0, "attention: token sets must tile [0, L)");
    m.start[i] = starts[i];
    m.len[i] = lens[i];
    m.vis[i] = vis[i] & ((1u << MAX_SETS) - 1u);
    m.causal |= ((vis[i] >> 31) & 1u) << i;   // MMT_SET_CAUSAL
    expect += lens[i];
  }
  MMT_CHECK_ARG(expect == L, "attention: token sets cover %d of L=%d", expect, L);
  for (int i = n_sets; i < MAX_SETS; ++i) {
    m.start[i] = 1 << 30;
    m.len[i] = 0;
    m.vis[i] = 0;
  }
  return MMT_OK;
}

}  // namespace

static int attn_cu_count() {
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

// forward query blocks per wave (0: automatic); MMT_ATTN_NQ=1..2 forces it (benchmarks)
static const int g_attn_nq = getenv("MMT_ATTN_NQ") ? atoi(getenv("MMT_ATTN_NQ")) : 0;
// the K/V-resident forward for Dh 64, 32 < L <= 320 (MMT_ATTN_RES=0: the streaming kernel;
// read per call so one process can A/B both)
static bool attn_res_enabled(const char* var = "MMT_ATTN_RES") {
  const char* e = getenv(var);
  return !e || atoi(e) != 0;
}

#define ATTN_DISPATCH(DH_, ...)                                  \
  do {                                                           \
    if (Dh == 64) { constexpr int DH_ = 64; __VA_ARGS__; }       \
    else if (Dh == 128) { constexpr int DH_ = 128; __VA_ARGS__; } \
    else if (Dh == 256) { constexpr int DH_ = 256; __VA_ARGS__; } \
    else { MMT_CHECK_ARG(false, "attention: head dim %d unsupported (64, 128, 256)", Dh); } \
  } while (0)

// Backward workgroup size: 2 waves (64 rows) when that fills the row blocks clearly better than
// 4 waves (128 rows) — measured at B = 256, Dh = 64: L = 292 398 -> 380 us, L = 132 177 -> 138 us,
// L = 212 (equal fill) 234 -> 257 us, so the smaller blocks must gain > 10 % fill.
inline int bwd_threads(int L) {
  static const int forced = getenv("MMT_ATTN_BWD_NT") ? atoi(getenv("MMT_ATTN_BWD_NT")) : 0;
  if (forced == 128 || forced == 256) return forced;  // (benchmarks)
  const double f128 = (double)L / (((L + 127) / 128) * 128);
  const double f64 = (double)L / (((L + 63) / 64) * 64);
  return f64 > f128 + 0.10 ? 128 : 256;
}

#define ATTN_BWD_LAUNCH2(DH_, NTT_, DR_)                                                          \
  do {                                                                                            \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<DH_, NTT_, DR_>), grid, dim3(NTT_), 0, s, g, m,        \
                       drop_bits, lp, dscale, (const bf16_t*)dout, d_s_b, d_s_t, lse,             \
                       (const bf16_t*)o, o_s_b, o_s_t, delta, (bf16_t*)dqkv, dq_s_b, dq_s_t,      \
                       bias_grad);                                                                \
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<DH_, NTT_, DR_>), grid, dim3(NTT_), 0, s, g, m,      \
                       drop_bits_t, lp, dscale, (const bf16_t*)dout, d_s_b, d_s_t, lse, delta,    \
                       (bf16_t*)dqkv, dq_s_b, dq_s_t, bias_grad);                                 \
  } while (0)
#define ATTN_BWD_LAUNCH(DH_, NTT_)                     \
  do {                                                 \
    if (drop_bits) ATTN_BWD_LAUNCH2(DH_, NTT_, true);  \
    else ATTN_BWD_LAUNCH2(DH_, NTT_, false);           \
  } while (0)

#if MMT_RES_ABL == 9
extern "C" int mmt_res8_stamps(void* dst, int64_t bytes) {
  const int64_t n = (int64_t)sizeof(g_res8_stamps);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_res8_stamps), bytes < n ? bytes : n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int mmt_dropout_bits(const uint32_t* rng, uint32_t layer, uint32_t site, int rows,
                                int cols, float keep_prob, uint32_t* out, uint32_t* out_t,
                                mmt_stream_t stream) {
  MMT_CHECK_ARG(rng && out && rows > 0 && cols > 0 && keep_prob > 0.f && keep_prob <= 1.f,
                "mmt_dropout_bits: bad args");
  MMT_CHECK_ARG(!out_t || rows == cols, "mmt_dropout_bits: the transposed mask needs rows == cols");
  const int words = (cols + 31) / 32;
  const int64_t n = out_t ? 2 * (int64_t)words * lp_of(rows) : (int64_t)rows * words;
  hipLaunchKernelGGL(dropout_bits_kernel, dim3((n + 255) / 256), dim3(256), 0, as_stream(stream),
                     rng, layer, site, rows, cols, words, keep_threshold16(keep_prob), out, out_t);
  MMT_CHECK_LAUNCH("mmt_dropout_bits");
  return MMT_OK;
}

extern "C" int mmt_attn_fwd(const void* qkv, int64_t s_b, int64_t s_t, int B, int L, int H, int Dh,
                            float scale, int n_sets, const int32_t* set_start,
                            const int32_t* set_len, const uint32_t* set_vis,
                            const uint32_t* drop_bits, float keep_prob, const float* bias,
                            void* o, int64_t o_s_b, int64_t o_s_t, float* lse, float* wsum,
                            mmt_stream_t stream) {
  MMT_CHECK_ARG(qkv && o && lse, "mmt_attn_fwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L > 0 && H > 0 && L <= MAXL, "mmt_attn_fwd: bad shape (L <= %d)", MAXL);
  MMT_CHECK_ARG(s_t % 8 == 0 && s_b % 8 == 0 && o_s_t % 4 == 0 && o_s_b % 4 == 0,
                "mmt_attn_fwd: strides must keep 16-B rows");
  MMT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "mmt_attn_fwd: keep_prob");
  MMT_CHECK_ARG(!bias || L % 4 == 0, "mmt_attn_fwd: the additive bias needs L %% 4 == 0 (float4 rows)");
  AttnMask m;
  int rc = fill_mask(m, n_sets, set_start, set_len, set_vis, L);
  if (rc) return rc;
  Geo g{(const bf16_t*)qkv, s_b, s_t, L, H, scale};
  const int lp = lp_of(L);
  const float dscale = drop_bits ? 1.f / keep_prob : 1.f;
  // query blocks per wave (Dh 64): two when one workgroup then covers L (K/V read once per
  // (b, h)); beyond 256 rows one (3 blocks per wave spill registers; measured at B = 256:
  // L = 292 117.6 / 150.5 / 122.6 us for 1 / 2 / 3 blocks, L = 212 73.1 / 71.5 / 78.2,
  // L = 132 48.1 / 44.0 / 48.8). Dh 128 / 256 keep one (registers).
  if (attn_res_enabled() && Dh == 64 && !bias && L > 32 && L <= 32 * RES_TILES) {
    ResPlan plan;
    if (res_plan(m, L, plan)) {
      const int ntile = ((L + 63) / 64) * 2;  // even tile counts are instantiated
      const bool one1 = attn_res_enabled("MMT_ATTN_ONEPASS");
#define RES1(NT_, DR_, WS_)                                                                       \
  do {                                                                                            \
    if (one1)                                                                                     \
      hipLaunchKernelGGL((attn_fwd_res_kernel<NT_, DR_, WS_, true>), dim3(B * H), dim3(64 * RES_NW), \
                         0, as_stream(stream), g, m, plan, drop_bits, lp, dscale, (bf16_t*)o, o_s_b, \
                         o_s_t, lse, wsum);                                                       \
    else                                                                                          \
      hipLaunchKernelGGL((attn_fwd_res_kernel<NT_, DR_, WS_, false>), dim3(B * H), dim3(64 * RES_NW), \
                         0, as_stream(stream), g, m, plan, drop_bits, lp, dscale, (bf16_t*)o, o_s_b, \
                         o_s_t, lse, wsum);                                                       \
  } while (0)
#define RES2(NT_)                                          \
  do {                                                     \
    if (drop_bits) {                                       \
      if (wsum) RES1(NT_, true, true);                     \
      else RES1(NT_, true, false);                         \
    } else {                                               \
      if (wsum) RES1(NT_, false, true);                    \
      else RES1(NT_, false, false);                        \
    }                                                      \
  } while (0)
      switch (ntile) {
        case 2: RES2(2); break;
        case 4: RES2(4); break;
        case 6: RES2(6); break;
        case 8: RES2(8); break;
        default: RES2(10); break;
      }
#undef RES2
#undef RES1
      MMT_CHECK_LAUNCH("mmt_attn_fwd");
      return MMT_OK;
    }
  }
  // (past the K/V-resident kernel's L <= 320 the tiled kernel also takes two blocks: OCTO-base,
  // B = 32, H = 12, tools/attn_bench.py: L = 1064 352.7 -> 312.5 us, L = 788 231.0 -> 193.1,
  // L = 532 114.3 -> 111.1)
  int nq = g_attn_nq > 0 ? std::min(g_attn_nq, 2) : (L <= 32 ? 1 : L <= 2 * QB ? 2 : L > 32 * RES_TILES ? 2 : 1);
  if (Dh > 64) nq = 1;
  dim3 grid((L + QB * nq - 1) / (QB * nq), H, B);
#define FWD1(DH_, NQ_, WS_, DR_)                                                                 \
  do {                                                                                            \
    bool one_wave = false;                                                                        \
    if constexpr (DH_ <= 64 && NQ_ == 1) {                                                        \
      if (L <= 32) { /* one 32-row block (the T5 text): one-wave workgroups */                    \
        one_wave = true;                                                                          \
        hipLaunchKernelGGL((attn_fwd_kernel<DH_, NQ_, WS_, DR_, 1>), dim3(1, H, B), dim3(64), 0,  \
                           as_stream(stream), g, m, drop_bits, lp, dscale, bias, (bf16_t*)o,      \
                           o_s_b, o_s_t, lse, wsum);                                              \
      }                                                                                           \
    }                                                                                             \
    if (!one_wave)                                                                                \
      hipLaunchKernelGGL((attn_fwd_kernel<DH_, NQ_, WS_, DR_>), grid, dim3(NT), 0,                \
                         as_stream(stream), g, m, drop_bits, lp, dscale, bias, (bf16_t*)o, o_s_b,  \
                         o_s_t, lse, wsum);                                                       \
  } while (0)
#define FWD(DH_, NQ_)                                          \
  do {                                                         \
    if (drop_bits) {                                           \
      if (wsum) FWD1(DH_, NQ_, true, true);                    \
      else FWD1(DH_, NQ_, false, true);                        \
    } else {                                                   \
      if (wsum) FWD1(DH_, NQ_, true, false);                   \
      else FWD1(DH_, NQ_, false, false);                       \
    }                                                          \
  } while (0)
  if (Dh == 64) {
    if (nq == 2) FWD(64, 2);
    else FWD(64, 1);
  } else {
    ATTN_DISPATCH(DH, FWD(DH, 1));
  }
#undef FWD
#undef FWD1
  MMT_CHECK_LAUNCH("mmt_attn_fwd");
  return MMT_OK;
}

extern "C" int mmt_attn_bwd(const void* qkv, int64_t s_b, int64_t s_t, int B, int L, int H, int Dh,
                            float scale, int n_sets, const int32_t* set_start,
                            const int32_t* set_len, const uint32_t* set_vis,
                            const uint32_t* drop_bits, const uint32_t* drop_bits_t,
                            float keep_prob, const void* o, int64_t o_s_b, int64_t o_s_t,
                            const void* dout, int64_t d_s_b, int64_t d_s_t, const float* lse,
                            float* delta, void* dqkv, int64_t dq_s_b, int64_t dq_s_t,
                            float* bias_grad, mmt_stream_t stream) {
  MMT_CHECK_ARG(qkv && o && dout && lse && delta && dqkv, "mmt_attn_bwd: null pointer");
  MMT_CHECK_ARG(B > 0 && L > 0 && H > 0 && L <= MAXL, "mmt_attn_bwd: bad shape");
  MMT_CHECK_ARG(s_t % 8 == 0 && d_s_t % 8 == 0 && dq_s_t % 4 == 0 && o_s_t % 8 == 0,
                "mmt_attn_bwd: strides must keep 16-B rows");
  MMT_CHECK_ARG(keep_prob > 0.f && keep_prob <= 1.f, "mmt_attn_bwd: keep_prob");
  MMT_CHECK_ARG(!drop_bits == !drop_bits_t,
                "mmt_attn_bwd: dropout needs both the mask and its transpose (mmt_dropout_bits)");
  AttnMask m;
  int rc = fill_mask(m, n_sets, set_start, set_len, set_vis, L);
  if (rc) return rc;
  Geo g{(const bf16_t*)qkv, s_b, s_t, L, H, scale};
  const int lp = lp_of(L);
  const float dscale = drop_bits ? 1.f / keep_prob : 1.f;
  hipStream_t s = as_stream(stream);
  if (attn_res_enabled("MMT_ATTN_RES_BWD") && Dh == 64 && L > 32 && L <= 32 * RES_TILES) {
    // the concurrent-phase kernel (MMT_ATTN_BWD8=0: the two-phase kernel; same dQ / dK / dV, bit
    // for bit). Alone (tools/attn_bench.py, B = 512) it wins at L = 292 (464 vs 516 us) and
    // L <= 164 (1.06-1.13x) and loses 0-6 % at L = 196 .. 276 (one workgroup per CU there);
    // in the step it is faster at every L (all: 14.75k, per-L choice: 14.73k, two-phase: 14.66k)
    const bool bwd8 = attn_res_enabled("MMT_ATTN_BWD8") &&
                      res8_need(L, ((L + 63) / 64) * 2) <= res8_lds(((L + 63) / 64) * 2);
    ResPlanB plan;
    if (bwd8 ? res_plan_bwd(m, L, plan, RES8_NA, 2 * RES_NW - RES8_NA) : res_plan_bwd(m, L, plan)) {
      // the work list at 192 < L <= 256 (tools/attn_bench.py B = 512, backward: L = 228 291 vs
      // 311 us with the static deal; L = 292 458 vs 452, L = 164 200 vs 194, so not there), not
      // in deterministic mode (its bias partials must not depend on which wave took a block);
      // MMT_ATTN_BWD8_DEAL=1: the static deal everywhere (A/B)
      static const bool deal = getenv("MMT_ATTN_BWD8_DEAL") && atoi(getenv("MMT_ATTN_BWD8_DEAL")) == 1;
      if (bwd8 && !deal && g_det_host.fx == nullptr && ((L + 63) / 64) * 2 == 8) res8_items(m, L, plan);
      const int ntile = ((L + 63) / 64) * 2;
#define RESB1(NT_, DR_)                                                                             \
  do {                                                                                              \
    if (bwd8)                                                                                       \
      hipLaunchKernelGGL((attn_bwd_res8_kernel<NT_, DR_>), dim3(B * H), dim3(128 * RES_NW), 0, s, g, \
                         m, plan, drop_bits, drop_bits_t, lp, dscale, (const bf16_t*)dout, d_s_b,   \
                         d_s_t, lse, (const bf16_t*)o, o_s_b, o_s_t, delta, (bf16_t*)dqkv, dq_s_b, \
                         dq_s_t, bias_grad);                                                        \
    else                                                                                            \
      hipLaunchKernelGGL((attn_bwd_res_kernel<NT_, DR_>), dim3(B * H), dim3(64 * RES_NW), 0, s, g,  \
                         m, plan, drop_bits, drop_bits_t, lp, dscale, (const bf16_t*)dout, d_s_b,   \
                         d_s_t, lse, (const bf16_t*)o, o_s_b, o_s_t, delta, (bf16_t*)dqkv, dq_s_b, \
                         dq_s_t, bias_grad);                                                        \
  } while (0)
#define RESB2(NT_)                  \
  do {                              \
    if (drop_bits) RESB1(NT_, true); \
    else RESB1(NT_, false);          \
  } while (0)
      switch (ntile) {
        case 2: RESB2(2); break;
        case 4: RESB2(4); break;
        case 6: RESB2(6); break;
        case 8: RESB2(8); break;
        default: RESB2(10); break;
      }
#undef RESB2
#undef RESB1
      MMT_CHECK_LAUNCH("mmt_attn_bwd");
      return MMT_OK;
    }
  }
  if (bwd_threads(L) == 128) {
    dim3 grid(((L + 63) / 64) * H * B);
    ATTN_DISPATCH(DH, ATTN_BWD_LAUNCH(DH, 128));
  } else {
    dim3 grid(((L + 127) / 128) * H * B);
    ATTN_DISPATCH(DH, ATTN_BWD_LAUNCH(DH, 256));
  }
  MMT_CHECK_LAUNCH("mmt_attn_bwd");
  return MMT_OK;
}

namespace mmt {
int det_set_attention(const DetState& st) { return det_set_unit(st); }
}  // namespace mmt
