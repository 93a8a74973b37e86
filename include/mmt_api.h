/* libmmt_hip — C ABI of the MI355X (gfx950) hot path of an OCTO-style multimodal transformer
 * training step with token merging (ToMe).
 *
 * The reference (maggieHao/multi_modal_transformers_TokenMerge, JAX/Flax) has no FFI: its
 * "interface" is the Flax module / function API. Each entry point below names the reference
 * function or Flax layer it replaces (paths relative to the reference's multi_modal_transformers/).
 *
 * Conventions
 *   - All tensor arguments are caller-owned DEVICE pointers; the library allocates nothing.
 *   - Strides are in ELEMENTS. Shapes are int, strides int64_t.
 *   - Every call is ordered on `stream` (a hipStream_t passed as void*), is graph-capturable
 *     (no host sync, no allocation) and returns MMT_OK (0) or a negative MMT_ERR_* code.
 *   - mmt_last_error() returns a thread-local description of the last failure.
 *   - dtype codes: MMT_F32 = 0, MMT_BF16 = 1.
 */
#ifndef MMT_API_H
#define MMT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mmt_stream_t;

enum { MMT_OK = 0, MMT_ERR_INVALID = -1, MMT_ERR_HIP = -2, MMT_ERR_UNSUPPORTED = -3 };
enum { MMT_F32 = 0, MMT_BF16 = 1 };
/* ToMe flags. CLASS/DISTILL: token_compression.py:57-64. PLAIN_SUM: the bare merge(x, "sum")
 * closure (no size weighting, no division). NO_SCATTER: merge(x, mode) with mode != "sum", which
 * in the reference leaves dst unchanged (:99-101). */
enum {
  MMT_TOME_CLASS_TOKEN = 1,
  MMT_TOME_DISTILL_TOKEN = 2,
  MMT_TOME_PLAIN_SUM = 4,
  MMT_TOME_NO_SCATTER = 8
};

const char* mmt_last_error(void);
/* ABI version of this header. 2: mmt_epilogue_t gained its trailing keep_bits field (a caller
 * built against version 1 passes a shorter struct: mmt_gemm would read past it). Callers check
 * mmt_version() == MMT_API_VERSION at load time and zero-initialise every mmt_epilogue_t
 * (memset / `= {0}`) before setting the fields they use, so fields added later read as unused. */
#define MMT_API_VERSION 2
int mmt_version(void);

/* Device-side index checks. The entry points that address memory through caller-supplied index
 * arrays (mmt_tome_merge_wavg_fwd / _bwd, mmt_tome_merge_seqnorm_fwd, mmt_ln_unmerge_dropout_bwd,
 * mmt_gather_rows, mmt_topk_scatter_bwd) cannot see those device values at launch. Their kernels
 * range-check every index they use; an invalid one is replaced by 0 (so no access leaves its
 * tensor and the context survives) and sets a bit of a library-wide device status word:
 *   MMT_FAULT_TOME_INDEX     unm / src not in [0, ceil(t/2)), dst not in [0, t/2)
 *   MMT_FAULT_TOME_PARTITION unm and src repeat an a-token (not a partition of the a half)
 *   MMT_FAULT_POS_MAP        pos_map entry not in [0, t - r)
 *   MMT_FAULT_ROW_INDEX      gathered / scattered row not in [0, L)
 * mmt_device_status synchronises `stream`, returns MMT_OK if the word is clear, else clears it and
 * returns MMT_ERR_INVALID with the decoded bits in mmt_last_error(). Not graph-capturable (it
 * synchronises); call it after a step, a test or a bench. The reference's jnp gathers cannot fault
 * (XLA clamps), so this adds the check the C ABI needs to keep its "never abort" convention. */
enum {
  MMT_FAULT_TOME_INDEX = 1,
  MMT_FAULT_TOME_PARTITION = 2,
  MMT_FAULT_POS_MAP = 4,
  MMT_FAULT_ROW_INDEX = 8
};
int mmt_device_status(mmt_stream_t stream);

/* Deterministic mode (SURVEY §5 "deterministic-mode reruns"). The gradient accumulations that are
 * otherwise fp32 atomics (bias / LayerNorm / GroupNorm / embedding / Fourier gradients, the
 * attention's QKV bias sums) go, for addresses inside the registered fp32 gradient buffer
 * [grad, grad + n), to fx: a signed 64-bit fixed-point shadow of it (round(v * 2^36), integer
 * atomics: order-independent). mmt_det_flush then adds fx * 2^-36 into grad and clears fx, so a
 * step's gradients are bitwise reproducible. fx NULL turns the mode off. mmt_set_deterministic is
 * synchronous: call it outside stream capture; fx must be zero-initialised. Replaces nothing in
 * the reference (its XLA reductions are deterministic per backend); reproducibility only. */
int mmt_set_deterministic(float* grad, long long* fx, int64_t n);
int mmt_det_flush(float* grad, long long* fx, int64_t n, mmt_stream_t stream);

/* Bytes of caller-provided device workspace an entry point needs (the library
 * allocates nothing; scratch comes from the caller). op / dims:
 *   MMT_WS_TOME_MATCH  {n, t, c}  (mmt_tome_match)
 * Returns the byte count, or a negative MMT_ERR_* code. */
enum { MMT_WS_TOME_MATCH = 1 };
int64_t mmt_workspace_size(int op, const int64_t* dims, int ndims);

/* ------------------------------------------------------------------ ToMe
 * mmt_tome_match replaces tokenizers/token_compression.py:54-112 (bipartite_soft_matching)
 * for an r that the caller has already clamped to min(r, (t - protected) // 2) > 0
 * (token_compression.py:66-70; the r <= 0 "do nothing" branch is the caller's).
 *
 * metric element (b, i, h, k) lives at metric[b*s_n + i*s_t + h*s_h + k]; the matching metric is
 * the fp32 sum over h = 0..heads-1 (heads = 1 for a plain (n, t, c) metric; heads = H gives the
 * ToMe key metric  sum_h K  of tome_attention.py:253).
 * Outputs (int32, per batch row contiguous): unm_idx[n][ta - r], src_idx[n][r], dst_idx[n][r],
 * where ta = ceil(t/2) (indices into the a = x[::2] / b = x[1::2] halves, exactly as the
 * reference's edge_idx / node_idx). node_max[n][ta] (fp32) is optional (may be NULL).
 * Arithmetic is canonical (see DESIGN.md "ToMe canonical arithmetic") so indices are bit-exact
 * with oracle/tome_ref.c. t <= 2048, c <= 512. workspace: >= mmt_workspace_size(
 * MMT_WS_TOME_MATCH, {n, t, c}) bytes, 16-B aligned (normalised metric halves, node_max/idx).
 */
int mmt_tome_match(const void* metric, int dtype, int n, int t, int heads, int c, int64_t s_n,
                   int64_t s_t, int64_t s_h, int r, int flags, int32_t* unm_idx, int32_t* src_idx,
                   int32_t* dst_idx, float* node_max, void* workspace, int64_t ws_bytes,
                   mmt_stream_t stream);

/* mmt_tome_merge_wavg_fwd replaces token_compression.py:114-129 (merge_wavg) applied with the
 * merge closure of :90-109 (mode "sum"), fused with the surrounding sequence copy:
 * x is a sequence (n, L, D) whose rows [set_start, set_start + t) are the merged token set; the
 * output sequence (n, L - r, D) holds rows [0, set_start) copied, then the t - r merged rows
 * (concat[unm, dst], or the distill interleave), then the remaining rows copied.
 * size_in (n, t) fp32 may be NULL (= ones). size_out (n, t - r) receives the merged sizes.
 * pos_map (n, t) int32 (optional) receives, for each set token, the merged row it went to.
 */
int mmt_tome_merge_wavg_fwd(const void* x, int dtype, int n, int L, int D, int64_t x_s_n,
                            int64_t x_s_t, int set_start, int t, int r, int flags,
                            const float* size_in, const int32_t* unm_idx, const int32_t* src_idx,
                            const int32_t* dst_idx, void* x_out, int64_t o_s_n, int64_t o_s_t,
                            float* size_out, int32_t* pos_map, mmt_stream_t stream);

/* Selects the score path of mmt_tome_match: 1 = f32 MFMA (v_mfma_f32_32x32x2_f32, default),
 * 0 = VALU fmaf chain. Both produce the same canonical fmaf chain; the switch exists so the
 * parity tests can check each against the oracle. */
void mmt_tome_set_match_path(int use_mfma);

/* Backward of mmt_tome_merge_wavg_fwd w.r.t. x (sizes carry no gradient; the metric carries
 * none either: argmax/argsort):  g_in[row] = g_out[pos(row)] * size_in[row] / size_out[pos(row)]
 * for set rows, plain copy for the others.  pos_map comes from the forward. size_in and size_out
 * may both be NULL: the bare merge(x, "sum") closure, whose Jacobian is a 0/1 gather. */
/* The backward of the same pair plus the attention-output dropout, fused: mmt_seqnorm_bwd over the
 * merged sequence (dy bf16, x and addend fp32, L2 = L - r rows), then mmt_tome_merge_wavg_bwd
 * (pos_map, size_in, size_out) into g_in (B, L, D) fp32, then mmt_dropout_bwd (layer, site,
 * keep_prob, row_offset; rng NULL = no dropout) of g_in into z bf16 with its column sums added
 * to bias_grad. The merged gradient stays in LDS. L <= 512, L2 * 256 B <= 96 KB. */
int mmt_ln_unmerge_dropout_bwd(const void* dy, int64_t ds_b, int64_t ds_t, const float* x,
                               int64_t xs_b, int64_t xs_t, int B, int L2, int D, const float* mean,
                               const float* rstd, const float* gamma, const float* addend,
                               int64_t as_b, int64_t as_t, float* dgamma, float* dbeta, int L,
                               int set_start, int t, int r, const float* size_in,
                               const float* size_out, const int32_t* pos_map, float* g_in,
                               int64_t gs_b, int64_t gs_t, const uint32_t* rng, uint32_t layer,
                               uint32_t site, float keep_prob, int64_t row_offset, void* z,
                               int64_t zs_b, int64_t zs_t, float* bias_grad, mmt_stream_t stream);
/* mmt_tome_merge_wavg_fwd fused with the sequence-axis LayerNorm forward that follows it in the
 * block (attention.py:66; mmt_seqnorm_fwd semantics): fp32 x, merged rows x_out (bit-identical to
 * the unfused merge), size_out / pos_map as there, y = LN(x_out) bf16 with mean / rstd (B, D)
 * (bit-identical to mmt_seqnorm_fwd on x_out). L - r <= 512, D % 8 == 0. */
int mmt_tome_merge_seqnorm_fwd(const float* x, int n, int L, int D, int64_t x_s_n, int64_t x_s_t,
                               int set_start, int t, int r, int flags, const float* size_in,
                               const int32_t* unm_idx, const int32_t* src_idx,
                               const int32_t* dst_idx, float* x_out, int64_t o_s_n, int64_t o_s_t,
                               float* size_out, int32_t* pos_map, const float* gamma,
                               const float* beta, float eps, void* y, int64_t y_s_n, int64_t y_s_t,
                               float* mean, float* rstd, mmt_stream_t stream);
int mmt_tome_merge_wavg_bwd(const void* g_out, int dtype, int n, int L, int D, int64_t go_s_n,
                            int64_t go_s_t, int set_start, int t, int r, const float* size_in,
                            const float* size_out, const int32_t* pos_map, void* g_in,
                            int64_t gi_s_n, int64_t gi_s_t, mmt_stream_t stream);


/* ------------------------------------------------------------------ top-k token pruning
 * mmt_topk_gather replaces tokenizers/token_compression.py:15-46 (compute_top_k_tokens, vmapped
 * over the batch, :168): for each token set s (host arrays set_start/set_len/set_k, <= 16 sets,
 * len <= 4096), the indices of jax.lax.top_k(scores[b, start:start+len], k) (descending, equal
 * scores keep the lower index first, float total order with NaN largest) + start, concatenated
 * over the sets in the given order -> idx_out (B, K = sum k) int32, and out[b, i] = x[b, idx].
 * x/out: (B, L, D) / (B, K, D) rows of fp32 or bf16 (dtype), 16-B aligned rows. */
int mmt_topk_gather(const void* x, int dtype, int B, int L, int D, int64_t xs_b, int64_t xs_t,
                    const float* scores, int64_t ss_b, int n_sets, const int32_t* set_start,
                    const int32_t* set_len, const int32_t* set_k, void* out, int64_t os_b,
                    int64_t os_t, int32_t* idx_out, mmt_stream_t stream);
/* out[b, i] = x[b, idx[b, i]] for i < K (rows of D fp32 / bf16 elements; idx (B, K) from
 * mmt_topk_gather): the residual stream of a pruned block follows its attention rows. */
int mmt_gather_rows(const void* x, int dtype, int B, int L, int D, int64_t xs_b, int64_t xs_t,
                    const int32_t* idx, int K, void* out, int64_t os_b, int64_t os_t,
                    mmt_stream_t stream);
/* Importance of compressed_attention.py:302-306 from mmt_attn_fwd's wsum: scores[b, q] =
 * (sum_h wsum[b, h, q] / L) / H (h ascending), the input of mmt_topk_gather. */
int mmt_prune_importance(const float* wsum, int B, int H, int L, float* scores, mmt_stream_t stream);
/* Backward of the gather: dx = 0, dx[b, idx[b, i]] = dout[b, i]. */
int mmt_topk_scatter_bwd(const void* dout, int dtype, int B, int K, int D, int64_t ds_b,
                         int64_t ds_t, const int32_t* idx, int L, void* dx, int64_t xs_b,
                         int64_t xs_t, mmt_stream_t stream);

/* ------------------------------------------------------------------ GEMM (MFMA bf16)
 * C = epilogue(op(A) . op(B)), fp32 accumulation, replacing every flax.linen.Dense /
 * DenseGeneral on the path (attention.py:32-37 MLPBlock; Flax SelfAttention q/k/v/out
 * projections configured in model_configs/attention_blocks/vanilla_decoder.yaml:19-31; the
 * image stem and output Dense, image_tokenizer.py:158-176; diffusion.py:41-65; T5 layers) and
 * their backward products (dX = dY.W, dW = dY^T.X).
 *   transA = 0: A is [M][K] (lda >= K);  transA = 1: A is stored [K][M] (lda >= M)
 *   transB = 0: B is [K][N] (ldb >= N);  transB = 1: B is stored [N][K] (ldb >= K)
 * A, B bf16; contiguous dims and strides multiples of 8 elements, base pointers 16-B aligned.
 * c_mode: MMT_OUT_BF16 (store), MMT_OUT_F32 (C = epi + beta*C), MMT_OUT_F32_ACCUM (C += alpha*acc,
 * the weight-gradient form; no other epilogue; with split_k > 1 the K range is split over
 * workgroups writing fp32 partial slabs into `workspace` (>= split_k*M*N floats, 16-B aligned)
 * which a second kernel sums into C — deterministic, no atomics).
 * Batched: blockIdx.z = batch index, with element strides sA, sB, sC.
 * N, ldc and sC must be multiples of 8 (8-column vector epilogue); A, B, C 16-B aligned.
 * Epilogue order: v = alpha*acc + bias[n]; act; v *= (gate[m][n] > 0 ? gate_scale : 0);
 * dropout (flax.linen.Dropout with a counter-based stream: element idx = (drop_row_offset + m)*N
 * + n keeps iff the 16-bit half (idx & 1) of mix32(key ^ (idx >> 1)) < floor(keep_prob * 65536),
 * key = stream_key(rng[0], rng[1], drop_layer, drop_site); kept values scaled by 1/keep_prob);
 * v += residual[m][n] (bf16 or fp32 per res_dtype).
 */
enum { MMT_ACT_NONE = 0, MMT_ACT_RELU = 1 };
#define MMT_SET_CAUSAL 0x80000000u
enum { MMT_OUT_BF16 = 0, MMT_OUT_F32 = 1, MMT_OUT_F32_ACCUM = 2 };

typedef struct {
  const float* bias;          /* [N] fp32 or NULL */
  int act;                    /* MMT_ACT_* */
  const uint32_t* rng;        /* device {seed, step} or NULL (no dropout) */
  uint32_t drop_layer, drop_site;
  float keep_prob;
  int64_t drop_row_offset;
  const void* gate;           /* bf16 [M][ld_gate] or NULL */
  int64_t ld_gate;
  float gate_scale;
  const void* residual;       /* [M][ld_res] bf16 or fp32 (res_dtype) or NULL */
  int64_t ld_res;
  float alpha, beta;
  int res_dtype;              /* MMT_BF16 / MMT_F32 */
  float* colsum;              /* [mmt_gemm_colsum_rows(...)][N] fp32 or NULL: row p = the column
                                 sums of C rows [256 p, 256 p + 256) as stored (bf16), written
                                 (not accumulated) — the bias gradient of the next Dense backward
                                 (layers.py:59 colsum) without re-reading C; only where
                                 mmt_gemm_colsum_rows is nonzero, else mmt_gemm fails */
  /* 1-bit form of the relu gate (the MLP hidden layer, attention.py:20-39 MLPBlock), both only
   * where mmt_gemm_colsum_rows is nonzero (the 256-wide bf16 NT path), else mmt_gemm fails:
   * relu_bits (out): [ceil(M/256)*256][N/32] words (16-B aligned), bit set iff the output is
   *   > 0 (the stored bf16 value has the same sign); output (m, n) is bit 8 c + e of the word
   *   at flat index (g * N/32 + w) * 4 + f, g = (m / 256) * 64 + ((m / 64) & 3) * 16 + (m & 15),
   *   f = (m / 16) & 3, n = 256 (w / 8) + 128 ((w / 4) & 1) + 8 (w & 3) + 32 c + e (c < 4,
   *   e < 8): one 16-B vector per lane of that path's epilogue (its 4 rows x 32 columns);
   * gate_bits (in): the same layout, used in place of gate (v *= bit ? gate_scale : 0), so a
   *   backward reads M*N/8 bytes instead of the bf16 gate's 2*M*N. NULL: unused.
   * keep_bits (in, relu_bits launches only, rng NULL): the dropout keep decisions in the same
   *   layout (mmt_gemm_dropout_keep_bits), applied as v = bit ? v / keep_prob : 0 in place of the
   *   counter-RNG draws — bit-identical outputs, the draws moved off the GEMM. NULL: unused. */
  uint32_t* relu_bits;
  const uint32_t* gate_bits;
  const uint32_t* keep_bits;
} mmt_epilogue_t;

/* Tuning knob (benchmarks): 0 = 128x128 register-staged, double-buffered LDS; 1 = same, single
 * LDS stage at 3 workgroups/CU; 2 = single stage with 128-deep K-steps; 3 = 256x192 tiles, 8
 * waves; 4 = direct-to-LDS (global_load_lds) 128x128 kernel for NT; -1 = automatic (default).
 * Process-wide, not thread-safe. */
void mmt_gemm_set_variant(int variant);
/* Rows of the epilogue's colsum slab for this launch shape (ceil(M / 256)), 0 when the kernel the
 * launch would use cannot write it (then take the column sums with mmt_colsum). */
int mmt_gemm_colsum_rows(int M, int N, int K, int transA, int transB, int c_mode, int split_k);
/* The keep_bits words of an (M, N) output's counter-RNG dropout (stream (rng, layer, site), rows
 * offset by row_offset: the draws mmt_gemm's epilogue would make with the same fields) into out
 * ([ceil(M/256)*256][N/32] words, 16-B aligned; N % 256 == 0). Replaces the per-element dropout
 * draws of the MLP hidden layer (attention.py:20-39 MLPBlock, nn.Dropout after the relu). */
int mmt_gemm_dropout_keep_bits(const uint32_t* rng, uint32_t layer, uint32_t site, int M, int N,
                               float keep_prob, int64_t row_offset, uint32_t* out, mmt_stream_t stream);
int mmt_gemm(int M, int N, int K, const void* A, int transA, int64_t lda, const void* B,
             int transB, int64_t ldb, void* C, int c_mode, int64_t ldc, int batch, int64_t sA,
             int64_t sB, int64_t sC, int split_k, const mmt_epilogue_t* epi, float* workspace,
             int64_t ws_elems, mmt_stream_t stream);

/* mmt_gemm_xs: C = X . W^T (+ bias[n]) in bf16 for the short-K products (K == 384: the
 * OCTO-small QKV projection), X [M][ldx], W [N][ldw] bf16, C [M][ldc] bf16, N % 64 == 0, 16-B
 * aligned rows; bias fp32 [N] or NULL. The activation-stationary kernel of csrc/gemm_xs.hip (a
 * 256-row panel of X held in registers while W streams through LDS); mmt_gemm routes its
 * K = 384 bf16 products with a bias / alpha / relu / dropout / relu_bits epilogue (M >= 32768;
 * relu_bits needs N % 256 == 0) and mmt_gemm_fp8 its K = 768 bf16-output products (no gate /
 * residual / relu_bits) there itself, with bit-identical outputs and bit images (reference
 * attention.py:20-37, 41-69 Dense layers). */
int mmt_gemm_xs(int M, int N, int K, const void* X, int64_t ldx, const void* W, int64_t ldw,
                void* C, int64_t ldc, const float* bias, mmt_stream_t stream);

/* FP8 weight path (BASELINE configs[4]; SURVEY §8c bar cosine >= 0.995): forward Dense products
 * in OCP e4m3 with one fp32 scale per activation row and per weight row (output channel).
 * mmt_quant_rows_fp8: scale[r] = amax|x[r,:]| / 448 (1 for a zero row), q[r,k] = e4m3(x[r,k] /
 * scale[r]) rounded to nearest even; x bf16 rows (stride ld), q uint8 rows (stride ldq), K % 8 == 0.
 * mmt_gemm_fp8: C = epilogue((A_q . B_q^T)[m][n] * sa[m] * sb[n]) with A_q [M][lda], B_q [N][ldb]
 * e4m3 (the NT form of mmt_gemm: B is the weight W[out][in]), on the block-scaled
 * v_mfma_scale_f32_32x32x64_f8f6f4 (unit block scales); same epilogue as mmt_gemm; c_mode
 * MMT_OUT_BF16 or MMT_OUT_F32. K % 64 == 0, N % 8 == 0, 16-B aligned rows. */
int mmt_quant_rows_fp8(const void* x, int64_t ld, int rows, int K, void* q, int64_t ldq,
                       float* scale, mmt_stream_t stream);
int mmt_gemm_fp8(int M, int N, int K, const void* A, int64_t lda, const float* sa, const void* B,
                 int64_t ldb, const float* sb, void* C, int c_mode, int64_t ldc,
                 const mmt_epilogue_t* epi, mmt_stream_t stream);

/* ------------------------------------------------------------------ attention
 * Blockwise-causal MHA replacing flax.linen.SelfAttention / dot_product_attention as the
 * reference configures it (vanilla_decoder.yaml:19-31, mask token_sequencer.py:313-321,
 * octo.py:66-68,119): softmax(where(mask, q.k * scale, finfo.min)) with attention dropout
 * sharing ONE (L, L) keep-mask across batch and heads (Flax broadcast_dropout) times v.
 * qkv: bf16 rows (b, t) at qkv + b*s_b + t*s_t holding [q(H,Dh) | k(H,Dh) | v(H,Dh)].
 * Mask = token-set table: n_sets (<= 16) contiguous sets tiling [0, L) (set_start/set_len HOST
 * arrays) and set_vis[s] = bitmask of key sets that query set s attends to; n_sets = 0: no mask.
 * Bit 31 of set_vis[s] (MMT_SET_CAUSAL) makes set s causal within itself: its query q sees its
 * own set's keys k <= q only (Text sets, token_sequencer.py:76-82, nn.make_causal_mask).
 * drop_bits: the query-word image of mmt_dropout_bits(.., L, L, ..) (its `out`), or NULL (no
 * dropout); kept probabilities are scaled by 1/keep_prob. bias: optional fp32 (H, L, L) added to the
 * scaled logits (T5 relative position bias; forward only). o: bf16 (b, t) rows of (H, Dh);
 * lse: fp32 (B, H, L) natural-log softmax normaliser. Dh in {64, 128, 256}.
 * wsum (optional, fp32 (B, H, L)): per query, the sum over keys of the attention weights AFTER
 * dropout (kept / keep_prob) — the per-head factor of the pruning importance score
 * (compressed_attention.py:302-306: mean over keys, then over heads; mmt_prune_importance).
 */
int mmt_attn_fwd(const void* qkv, int64_t s_b, int64_t s_t, int B, int L, int H, int Dh,
                 float scale, int n_sets, const int32_t* set_start, const int32_t* set_len,
                 const uint32_t* set_vis, const uint32_t* drop_bits, float keep_prob,
                 const float* bias, void* o, int64_t o_s_b, int64_t o_s_t, float* lse,
                 float* wsum, mmt_stream_t stream);
/* Backward: writes dq, dk, dv into dqkv (same row layout as qkv). delta: fp32 workspace of
 * B * H * 2 * roundup(L, 64) floats (rowsum(dO * O), and the row constants of the K/V-resident
 * kernel used for Dh 64 and 32 < L <= 320). drop_bits / drop_bits_t: the query-word and key-word images of
 * mmt_dropout_bits (`out` / `out_t`); both or neither. bias_grad (fp32 [3 H Dh], may be NULL) += the
 * column sums of dq | dk | dv over (B, L): the bias gradient of the fused QKV projection. */
int mmt_attn_bwd(const void* qkv, int64_t s_b, int64_t s_t, int B, int L, int H, int Dh,
                 float scale, int n_sets, const int32_t* set_start, const int32_t* set_len,
                 const uint32_t* set_vis, const uint32_t* drop_bits, const uint32_t* drop_bits_t,
                 float keep_prob, const void* o, int64_t o_s_b, int64_t o_s_t, const void* dout,
                 int64_t d_s_b, int64_t d_s_t, const float* lse, float* delta, void* dqkv,
                 int64_t dq_s_b, int64_t dq_s_t, float* bias_grad, mmt_stream_t stream);
/* Keep mask of a dropout stream (flax Dropout keep-mask, broadcast over batch and heads for
 * attention): keep(r, c) iff keep_elem(key(rng, layer, site), r*cols + c), i.e. the 16-bit half
 * (idx & 1) of mix32(key ^ (idx >> 1)) is below floor(keep_prob * 65536).
 * out_t == NULL: row-major words (rows, ceil(cols/32)), bit j of word (r, w) = keep(r, 32w + j).
 * out_t != NULL (attention, rows == cols == L): two word-major images of W = ceil(L/32) rows of
 * LP = roundup(L, 64) words, positions interleaved pos(8g + 4h + i) = 8g + 2i + h, zero past L:
 *   out   (query words): bit j of word (w, pos(k)) = keep(32w + j, k)
 *   out_t (key words):   bit j of word (w, pos(q)) = keep(q, 32w + j)
 * so that the 64-bit pair 16u + r of a 64-aligned tile's words is the wave lane mask of MFMA
 * accumulator register r of the tile's 32-wide half u (read into SGPRs by the attention kernels). */
int mmt_dropout_bits(const uint32_t* rng, uint32_t layer, uint32_t site, int rows, int cols,
                     float keep_prob, uint32_t* out, uint32_t* out_t, mmt_stream_t stream);

/* ------------------------------------------------------------------ sequence LayerNorm
 * flax.linen.LayerNorm(reduction_axes=[1], feature_axes=[-1], epsilon) as used in
 * attention.py:58,66 (vanilla_decoder.yaml:5-13): stats per (b, d) over the SEQUENCE axis L,
 * fast variance; x (B, L, D) strided, bf16 or fp32 (x_dtype; the training path keeps the residual
 * stream in fp32 because this normalisation subtracts a large per-feature sequence mean); y bf16;
 * mean/rstd fp32 (B, D) saved for the backward. */
int mmt_seqnorm_fwd(const void* x, int x_dtype, int64_t xs_b, int64_t xs_t, int B, int L, int D,
                    const float* gamma, const float* beta, float eps, void* y, int64_t ys_b,
                    int64_t ys_t, float* mean, float* rstd, mmt_stream_t stream);
/* dx = LN backward (+ addend, which may alias dx); x, addend and dx have x_dtype, dy has
 * dy_dtype; dgamma/dbeta fp32 [D] are ACCUMULATED. */
int mmt_seqnorm_bwd(const void* dy, int dy_dtype, int64_t ds_b, int64_t ds_t, const void* x,
                    int x_dtype, int64_t xs_b, int64_t xs_t, int B, int L, int D,
                    const float* mean, const float* rstd,
                    const float* gamma, const void* addend, int64_t as_b, int64_t as_t, void* dx,
                    int64_t dxs_b, int64_t dxs_t, float* dgamma, float* dbeta,
                    mmt_stream_t stream);
/* mmt_seqnorm_bwd (bf16 dy, fp32 x / addend / dx) that also applies the dropout backward of the
 * PREVIOUS block's MLP output (layer, site, keep_prob, row_offset; rng NULL = a plain cast) to
 * the dx it writes: z (B, L, D) bf16 = keep ? dx / keep_prob : 0, colsum += its column sums (as
 * mmt_dropout_bwd), without reading dx back. */
int mmt_seqnorm_dropout_bwd(const void* dy, int64_t ds_b, int64_t ds_t, const float* x,
                            int64_t xs_b, int64_t xs_t, int B, int L, int D, const float* mean,
                            const float* rstd, const float* gamma, const float* addend,
                            int64_t as_b, int64_t as_t, float* dx, int64_t dxs_b, int64_t dxs_t,
                            float* dgamma, float* dbeta, const uint32_t* rng, uint32_t layer,
                            uint32_t site, float keep_prob, int64_t row_offset, void* z,
                            int64_t zs_b, int64_t zs_t, float* colsum, mmt_stream_t stream);

/* ------------------------------------------------------------------ reductions / dropout
 * out[n] += sum_m x[m][n] (bf16 x, fp32 out): Dense bias gradients. */
int mmt_colsum(const void* x, int dtype, int64_t ldx, int M, int N, float* out,
               mmt_stream_t stream);
/* Backward of a GEMM-epilogue dropout (flax.linen.Dropout, attention.py:34-37,60):
 * dz = dy * keep / keep_prob (bf16) with the same stream/counters as the forward (rng NULL:
 * keep everything — a cast); colsum (optional) += column sums of dz (the bias gradient of the
 * Dense before the dropout). dy: bf16 or fp32 (dtype). */
int mmt_dropout_bwd(const void* dy, int dtype, int64_t ldy, int M, int N, const uint32_t* rng,
                    uint32_t layer, uint32_t site, float keep_prob, int64_t row_offset, void* dz,
                    int64_t ldz, float* colsum, mmt_stream_t stream);

/* ------------------------------------------------------------------ image tokenizer stem
 * tokenizers/images/image_tokenizer.py: image_to_patches (:35-71, raster "(h p1)(w p2) -> (h w)",
 * normalise 2*(x/255)-1) fused with the im2col of the input Conv (KHxKW stride S VALID, Flax HWIO
 * kernel order (ky, kx, c)), :158. img: (B, I, H, H, C) fp32 (in_dtype 0) or uint8 (in_dtype 2);
 * out: bf16 [B*I*NP*OH*OW][KH*KW*C]. H % P != 0 is rejected (the reference's resize branch,
 * :54-59, is broken). */
int mmt_patch_im2col(const void* img, int in_dtype, int B, int I, int Himg, int C, int P, int KH,
                     int KW, int S, int normalize, void* out, mmt_stream_t stream);
/* max_pool over the `win` conv outputs of each patch (3x3 s1 VALID on the 3x3 map, :159) with
 * first-max argmax for the backward (fp32 conv [npatch][win][C] -> fp32 pooled [npatch][C]);
 * the backward scatters fp32 dpooled into the bf16 conv-output gradient G [npatch][win][C]. */
/* The stem's input conv and pool fused (image_tokenizer.py:35-71,140-162 at its gato_resnet
 * configuration): for every 16x16 patch of uint8 RGB images (B, I, H, H, 3), normalised as
 * 2 * (x / 255) - 1, the 12x12 stride-2 VALID conv with w (64, 432) bf16 [out][(ky, kx, c)] plus
 * bias, then the max over its 3x3 map: pooled (B*I*NP, 64) fp32 and the first-maximum position
 * argmax (B*I*NP, 64) uint8 (as mmt_maxpool_patch), without the im2col matrix. */
int mmt_stem_conv_pool(const void* img, int B, int I, int Himg, const void* w, const float* bias,
                       float* pooled, uint8_t* argmax, mmt_stream_t stream);
/* Its weight gradient without im2col: dw (64, 432) += sum over patches and conv positions of
 * G^T A, G the max-pool backward of dpooled (B*I*NP, 64) fp32 at argmax (bf16-rounded, as
 * mmt_maxpool_patch_bwd), A the normalised patch pixels: each of mmt_stem_conv_wgrad_slabs(B, I,
 * Himg) workgroups writes its partial (64, 432) to slab row i (caller-owned fp32), which the
 * caller sums into dw (mmt_colsum). */
int mmt_stem_conv_wgrad_slabs(int B, int I, int Himg);
int mmt_stem_conv_wgrad(const void* img, int B, int I, int Himg, const float* dpooled,
                        const uint8_t* argmax, float* slab, int64_t slab_elems,
                        mmt_stream_t stream);
int mmt_maxpool_patch(const void* conv, int64_t npatch, int win, int C, void* pooled,
                      uint8_t* argmax, mmt_stream_t stream);
int mmt_maxpool_patch_bwd(const void* dpooled, const uint8_t* argmax, int64_t npatch, int win,
                          int C, void* G, mmt_stream_t stream);
/* General stem maps (pooled map larger than 1 x 1: the reference's patch 56, 23 x 23 conv map,
 * image_tokenizer.py:156-176 with gato_resnet.yaml:45-92):
 * max_pool KP x KP stride 1 VALID over (npatch, OH, OW, C) fp32 -> (npatch, OH-KP+1, OW-KP+1, C)
 * plus the first-maximum window slot; its backward writes the bf16 (npatch, OH, OW, C) operand of
 * the conv weight gradient (gather over the windows, deterministic). */
int mmt_maxpool2d(const void* x, int64_t npatch, int OH, int OW, int C, int KP, void* y,
                  uint8_t* argmax, mmt_stream_t stream);
int mmt_maxpool2d_bwd(const void* dy, const uint8_t* argmax, int64_t npatch, int OH, int OW, int C,
                      int KP, void* G, mmt_stream_t stream);
/* KS x KS stride-1 SAME convolution as im2col (bf16 (npatch, H, W, C) -> (npatch*H*W, KS*KS*C) in
 * Flax HWIO (ky, kx, c) order, zero padding) + GEMM; col2im sums the fp32 column gradient back. */
int mmt_im2col_same(const void* x, int64_t npatch, int H, int W, int C, int KS, void* cols,
                    mmt_stream_t stream);
int mmt_col2im_same(const float* dcols, int64_t npatch, int H, int W, int C, int KS, float* dx,
                    mmt_stream_t stream);
/* flax GroupNorm(num_groups=G, eps) over every non-batch axis + gelu(tanh approx)
 * (gato_resnet.yaml:77-86, image_tokenizer.py:165-167): x (B, R, C) fp32 -> y bf16 (the next
 * conv's GEMM operand); statistics in fp32. */
int mmt_groupnorm_gelu_fwd(const void* x, int B, int R, int C, int G, float eps,
                           const float* gamma, const float* beta, void* y, float* mean,
                           float* rstd, mmt_stream_t stream);
/* backward (dy, x, dx fp32); dx += result when accumulate != 0; dgamma/dbeta accumulated. */
int mmt_groupnorm_gelu_bwd(const void* dy, const void* x, int B, int R, int C, int G,
                           const float* gamma, const float* beta, const float* mean,
                           const float* rstd, void* dx, int accumulate, float* dgamma,
                           float* dbeta, mmt_stream_t stream);
/* encode_patch_position (:74-132) for every (b, image, patch): Q quantisation levels, row token
 * from interval p % PPD, col from p // PPD; train: randint[start, stop) on the counter stream keyed
 * by the global sample index (sample_offset + b); eval: (start + stop) // 2. */
int mmt_patch_positions(const uint32_t* rng, uint32_t site, int B, int I, int Himg, int P, int Q,
                        int train, int64_t sample_offset, int32_t* row_tok, int32_t* col_tok,
                        mmt_stream_t stream);

/* ------------------------------------------------------------------ sequence assembly
 * x0[b, l] = source(l) + pe[l] with source = text[b, j] | img[b, j] + row_emb[rtok] + col_emb[ctok]
 * | readout_pe[j]  (row_src[l] = kind << 24 | j, kind 0 text / 1 image / 2 readout):
 * TokenSequence.assemble_embeddings (token_sequencer.py:255-269), readout AddPositionEmbedding
 * on zeros (readout.py:18-33, octo.py:103-108), ImageTokenizer embeddings (:300-307) and the
 * encoder's learned position embedding (attention.py:71-85,97-100), fused. fp32 tables. */
int mmt_seq_assemble_fwd(int B, int L, int D, const int32_t* row_src, const void* text, int T,
                         const void* img, int NI, const int32_t* rtok, const int32_t* ctok,
                         const float* row_emb, const float* col_emb, const float* readout_pe,
                         const float* pe, void* x0, mmt_stream_t stream);
/* backward: gathers d(text), d(img) (bf16) from the fp32 dx0, accumulates d(readout_pe) and the
 * (Q, D) row/col embedding gradients (LDS histograms per 64-column slice, then one global
 * atomic per table entry). img_rows[j] = sequence row of image token j. d(pe) is mmt_colsum
 * over the batch. */
int mmt_seq_assemble_bwd(int B, int L, int D, const int32_t* row_src, const void* dx0,
                         void* dtext, int T, void* dimg, int NI, const int32_t* rtok,
                         const int32_t* ctok, const int32_t* img_rows, int Q, float* drow_emb,
                         float* dcol_emb, float* dreadout_pe, mmt_stream_t stream);
/* The image row / column position-embedding gradients alone (drow_emb = dcol_emb = NULL above):
 * d(row_emb)[t] += dx0[b, img_rows[j]] over the image tokens (b, j) whose row token (rtok, from
 * mmt_patch_positions) is t, likewise columns. A patch row's tokens lie in one window of the
 * table (patch_positions' q(ri P) .. q((ri + 1) P)), so a workgroup owns one window and keeps a
 * register accumulator per window token: no LDS atomics (the form above: 268 -> ~40 us per step
 * at OCTO-small B = 256). I images of Himg x Himg pixels, patch P, table Q rows per axis, dx0
 * fp32 (B, L, D), tables fp32 (Q, D) accumulated. */
int mmt_patch_embed_grad(int B, int L, int D, int I, int Himg, int P, int Q,
                         const int32_t* img_rows, const void* dx0, const int32_t* rtok,
                         const int32_t* ctok, float* drow_emb, float* dcol_emb,
                         mmt_stream_t stream);
/* AddPositionEmbedding standalone (tokenizers/readout/readout.py:18-33; also attention.py:71-85):
 * out (B, L, D) fp32 = x + pe[None] (x may alias out). Backward: dx = dout; d(pe) = mmt_colsum of
 * dout viewed as (B, L*D). The training step fuses this add into mmt_seq_assemble_fwd. */
int mmt_add_position_embedding(const float* x, const float* pe, float* out, int B, int L, int D,
                               mmt_stream_t stream);
/* readout gather + mean (octo.py:122-124, diffusion.py:102): out[b] = mean_i x[b, rows[i]]. */
int mmt_rows_mean_fwd(const void* x, int64_t xs_b, int64_t xs_t, int B, int D,
                      const int32_t* rows, int nrows, void* out, int64_t ld_out,
                      mmt_stream_t stream);
int mmt_rows_mean_bwd(const void* de, int64_t ld_de, int B, int L, int D, const int32_t* row_flag,
                      int nrows, void* dx, mmt_stream_t stream);

/* ------------------------------------------------------------------ diffusion head
 * DiffusionActionHead.denoise_loss (diffusion.py:110-143) pieces: t ~ U{0..steps-1}, eps ~ N(0,1)
 * (or injected), noisy = sqrt(abar_t) a + sqrt(1-abar_t) eps written to cat[:, :A] (bf16),
 * FourierFeatures (:41-51) [cos 2 pi t W, sin 2 pi t W] (bf16 (B, 2F)). */
int mmt_diffusion_prep(const uint32_t* rng, int B, int A, int steps, int64_t sample_offset,
                       const float* actions, const float* alpha_hats, const float* fourier_w,
                       int F, const int32_t* t_in, const float* eps_in, int32_t* t_out,
                       float* eps_out, void* cat, int64_t ld_cat, void* feats,
                       mmt_stream_t stream);
int mmt_fourier_bwd(const void* dfeats, int B, int F, const int32_t* t, const float* fourier_w,
                    float* dw, mmt_stream_t stream);
/* optax.l2_loss summed over actions, mean over batch; dpred = (pred-eps)*grad_scale/B (bf16). */
int mmt_diffusion_loss(const float* pred, int64_t ld_pred, const float* eps, int B, int A,
                       float grad_scale, float* loss, void* dpred, mmt_stream_t stream);
/* DiffusionActionHead.predict_action (diffusion.py:146-209), SURVEY §8f row 2: all `steps`
 * DDPM steps (t = steps-1 .. 0) in one launch, one wave per sample. The first denoiser Dense is
 * pre-split by the caller: P (B, H) fp32 = readout_mean . W1[:, A+T:]^T, Q (steps, H) fp32 =
 * time_emb(t) . W1[:, A:A+T]^T + b1; w1 is the bf16 W1 (row stride ld_w1, its first A columns
 * are read), w2 the bf16 (A, H) output kernel, b2 (A,), coef (steps, 3) = [1/sqrt(a_t),
 * (1-a_t)/sqrt(1-abar_t), sqrt(b_t)]. z_in (B, A) injects the initial sample (else drawn from the
 * counter stream keyed by rng and the global sample index); the same z is the noise of every step
 * (the reference never splits its keys, :178). A must be 8 (:200). Writes actions (B, A) fp32
 * and, if z_out is non-NULL, z (B, A). */
int mmt_diffusion_sample(const uint32_t* rng, int B, int A, int steps, int64_t sample_offset,
                         const float* P, int64_t ld_p, const float* Q, int64_t ld_q,
                         const void* w1, int64_t ld_w1, const void* w2, const float* b2,
                         const float* coef, const float* z_in, int H, float* actions,
                         float* z_out, mmt_stream_t stream);

/* Transposed bf16 weight shadows (this build's layout, no reference twin): for each of n
 * matrices, desc[5i..5i+4] = {src_off, dst_off, rows, cols, first_tile} (elements / 64x64 tiles,
 * first_tile = running tile count), dst[dst_off + c*rows + r] = src[src_off + r*cols + c]. */
int mmt_transpose_bf16_batched(const void* src, void* dst, const int64_t* desc, int n,
                               int64_t total_tiles, mmt_stream_t stream);

/* ------------------------------------------------------------------ continuous / categorical heads
 * (SURVEY §8f row 4). Grouped readout means (categorical.py:32-37): out (B, G, D) bf16 = mean of
 * the rows with row_group[l] == g (counts[g] rows); backward writes the whole fp32 dx (B, L, D). */
int mmt_rows_group_mean_fwd(const void* x, int64_t xs_b, int64_t xs_t, int B, int L, int D,
                            const int32_t* row_group, int G, const int32_t* counts, void* out,
                            mmt_stream_t stream);
int mmt_rows_group_mean_bwd(const void* de, int B, int L, int D, const int32_t* row_group, int G,
                            const int32_t* counts, void* dx, mmt_stream_t stream);
/* kind 0: ContinuousActionHead tanh squash (continuous.py:26) + compute_l2_loss (octo.py:167-174);
 * kind 1: CategoricalActionHead logits + compute_ce_loss with assign_bins (octo.py:187-198,
 * categorical.py:12-22: digitize over `edges`, one_hot(bin, N) zero past the last class).
 * loss (+=, zero it first) = inv_count x sum of the per-row losses; dz bf16 (R, N). y NULL:
 * forward only (kind 0 writes pred). */
int mmt_action_head(int kind, const float* z, int64_t ldz, int R, int N, const float* y,
                    const float* edges, int n_edges, float max_action, float inv_count, float* pred,
                    float* loss, void* dz, mmt_stream_t stream);

/* ------------------------------------------------------------------ T5 encoder pieces
 * (tokenizers/text/t5_base.py:8-15, frozen FlaxT5 encoder): T5LayerNorm and the shared
 * embedding lookup. */
int mmt_rmsnorm_fwd(const void* x, int64_t rows, int D, const void* w, float eps, void* y,
                    mmt_stream_t stream);
int mmt_embedding_gather(const int32_t* ids, int64_t n, int D, const void* table, int vocab,
                         void* out, mmt_stream_t stream);

/* ------------------------------------------------------------------ optimizer / state
 * Fused AdamW over the flat fp32 parameter buffer (the reference takes an optax tx from the
 * caller, octo.py:228,341; this is optax.adamw semantics), writing the bf16 shadow copy.
 * state = device {seed, step}: step+1 is the bias-correction count; mmt_step_advance
 * increments it (keys every random stream of the next step). Hyper-parameters in double (the
 * caller's Python floats): 1 - beta and the bias corrections are formed in double. */
int mmt_adamw(float* p, const float* g, float* m, float* v, void* shadow_bf16, int64_t n,
              const int32_t* state, double lr, double b1, double b2, double eps, double wd,
              float grad_scale, mmt_stream_t stream);
int mmt_cast_f32_bf16(const float* a, void* b, int64_t n, mmt_stream_t stream);
int mmt_step_advance(int32_t* state, mmt_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MMT_API_H */
