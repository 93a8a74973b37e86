"""Torch-facing wrappers of the C ABI (device tensors in, device tensors out).

Each wrapper validates shapes/dtypes/devices on the host BEFORE launching (a bad shape must never
reach a kernel) and calls exactly one libmmt_hip entry point on the current HIP stream. Nothing
here computes on the CPU: a missing library raises (see _C.py).
"""
from __future__ import annotations

import os

import torch

from . import _C
from ._C import ptr

DT = {torch.float32: 0, torch.bfloat16: 1}


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype not in DT:
        raise TypeError(f"unsupported dtype {t.dtype}; expected float32 or bfloat16")
    return DT[t.dtype]


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("libmmt_hip ops take device (cuda/HIP) tensors only")


def device_status() -> None:
    """Synchronise the current stream and raise MMTError if a kernel's device-side index check
    fired since the last call (mmt_device_status, include/mmt_api.h: ToMe merge maps, pos_map and
    gathered rows are range-checked on the GPU; an invalid index is replaced by 0 and recorded
    instead of faulting the context). Not capturable: call it after a step / graph replay."""
    _C.call("mmt_device_status", _C.stream_ptr())


# ------------------------------------------------------------------------------------ ToMe
FLAG_CLASS, FLAG_DISTILL, FLAG_PLAIN_SUM, FLAG_NO_SCATTER = 1, 2, 4, 8


def set_tome_match_path(use_mfma: bool) -> None:
    _C.call("mmt_tome_set_match_path", int(bool(use_mfma)))


def tome_match(metric: torch.Tensor, r: int, flags: int = 0, return_node_max: bool = False):
    """metric (n, t, c) or (n, t, heads, c) (any strides with unit inner stride) -> (unm, src, dst
    [, node_max]) int32 device tensors. r must already be clamped (> 0)."""
    _dev(metric)
    if metric.dim() == 3:
        n, t, c = metric.shape
        heads, s_h = 1, 0
        s_n, s_t = metric.stride(0), metric.stride(1)
        if metric.stride(2) != 1:
            raise ValueError("metric must have unit stride along c")
    elif metric.dim() == 4:
        n, t, heads, c = metric.shape
        s_n, s_t, s_h = metric.stride(0), metric.stride(1), metric.stride(2)
        if metric.stride(3) != 1:
            raise ValueError("metric must have unit stride along c")
    else:
        raise ValueError("metric must be (n, t, c) or (n, t, heads, c)")
    ta = (t + 1) // 2
    dev = metric.device
    unm = torch.empty((n, ta - r), dtype=torch.int32, device=dev)
    src = torch.empty((n, r), dtype=torch.int32, device=dev)
    dst = torch.empty((n, r), dtype=torch.int32, device=dev)
    nmax = torch.empty((n, ta), dtype=torch.float32, device=dev) if return_node_max else None
    ws = torch.empty(_C.workspace_size(_C.WS_TOME_MATCH, n, t, c), dtype=torch.uint8, device=dev)
    _C.call("mmt_tome_match", ptr(metric), _dtype_code(metric), n, t, heads, c, s_n, s_t, s_h, r,
            flags, ptr(unm), ptr(src), ptr(dst), ptr(nmax), ptr(ws), ws.numel(), _C.stream_ptr())
    return (unm, src, dst, nmax) if return_node_max else (unm, src, dst)


def tome_merge_fwd(x: torch.Tensor, set_start: int, t: int, r: int, unm, src, dst,
                   size_in: torch.Tensor | None = None, flags: int = 0, out: torch.Tensor | None = None,
                   want_pos_map: bool = True):
    """x (n, L, D) sequence; merges rows [set_start, set_start+t). Returns (x_out (n, L-r, D),
    size_out (n, t-r) fp32, pos_map (n, t) int32 or None)."""
    _dev(x, size_in, unm, src, dst)
    n, L, D = x.shape
    if x.stride(2) != 1:
        raise ValueError("x must have unit stride along D")
    if not (0 <= set_start and set_start + t <= L):
        raise ValueError("token set out of range")
    for a, shape in ((unm, (n, (t + 1) // 2 - r)), (src, (n, r)), (dst, (n, r))):
        if tuple(a.shape) != shape or a.dtype != torch.int32 or not a.is_contiguous():
            raise ValueError(f"index tensor must be contiguous int32 {shape}")
    if size_in is not None:
        if tuple(size_in.shape) != (n, t) or size_in.dtype != torch.float32 or not size_in.is_contiguous():
            raise ValueError("size_in must be contiguous fp32 (n, t)")
    if out is None:
        out = torch.empty((n, L - r, D), dtype=x.dtype, device=x.device)
    size_out = torch.empty((n, t - r), dtype=torch.float32, device=x.device)
    pos_map = torch.empty((n, t), dtype=torch.int32, device=x.device) if want_pos_map else None
    _C.call("mmt_tome_merge_wavg_fwd", ptr(x), _dtype_code(x), n, L, D, x.stride(0), x.stride(1),
            set_start, t, r, flags, ptr(size_in), ptr(unm), ptr(src), ptr(dst), ptr(out),
            out.stride(0), out.stride(1), ptr(size_out), ptr(pos_map), _C.stream_ptr())
    return out, size_out, pos_map


def tome_merge_seqnorm_fwd(x: torch.Tensor, set_start: int, t: int, r: int, unm, src, dst,
                           gamma: torch.Tensor, beta: torch.Tensor, eps: float,
                           size_in: torch.Tensor | None = None, flags: int = 0):
    """tome_merge_fwd (fp32 x) followed by seqnorm_fwd in one launch: returns (x_out, size_out,
    pos_map, y bf16, mean, rstd), each bit-identical to the two-launch form."""
    _dev(x, size_in, unm, src, dst, gamma, beta)
    n, L, D = x.shape
    if x.dtype != torch.float32 or x.stride(2) != 1:
        raise ValueError("tome_merge_seqnorm_fwd takes an fp32 (n, L, D) sequence, unit stride along D")
    if not (0 <= set_start and set_start + t <= L) or L - r > 512:
        raise ValueError("token set out of range or sequence too long for the fused form")
    for a, shape in ((unm, (n, (t + 1) // 2 - r)), (src, (n, r)), (dst, (n, r))):
        if tuple(a.shape) != shape or a.dtype != torch.int32 or not a.is_contiguous():
            raise ValueError(f"index tensor must be contiguous int32 {shape}")
    if size_in is not None and (tuple(size_in.shape) != (n, t) or size_in.dtype != torch.float32
                                or not size_in.is_contiguous()):
        raise ValueError("size_in must be contiguous fp32 (n, t)")
    out = torch.empty((n, L - r, D), dtype=torch.float32, device=x.device)
    size_out = torch.empty((n, t - r), dtype=torch.float32, device=x.device)
    pos_map = torch.empty((n, t), dtype=torch.int32, device=x.device)
    y = torch.empty((n, L - r, D), dtype=torch.bfloat16, device=x.device)
    mean = torch.empty((n, D), dtype=torch.float32, device=x.device)
    rstd = torch.empty((n, D), dtype=torch.float32, device=x.device)
    _C.call("mmt_tome_merge_seqnorm_fwd", ptr(x), n, L, D, x.stride(0), x.stride(1), set_start, t,
            r, flags, ptr(size_in), ptr(unm), ptr(src), ptr(dst), ptr(out), out.stride(0),
            out.stride(1), ptr(size_out), ptr(pos_map), ptr(gamma), ptr(beta), eps, ptr(y),
            y.stride(0), y.stride(1), ptr(mean), ptr(rstd), _C.stream_ptr())
    return out, size_out, pos_map, y, mean, rstd


def tome_merge_bwd(g_out: torch.Tensor, set_start: int, t: int, r: int, pos_map: torch.Tensor,
                   size_in: torch.Tensor | None, size_out: torch.Tensor | None,
                   out: torch.Tensor | None = None):
    _dev(g_out, pos_map, size_in, size_out)
    n, Lr, D = g_out.shape
    L = Lr + r
    if out is None:
        out = torch.empty((n, L, D), dtype=g_out.dtype, device=g_out.device)
    _C.call("mmt_tome_merge_wavg_bwd", ptr(g_out), _dtype_code(g_out), n, L, D, g_out.stride(0),
            g_out.stride(1), set_start, t, r, ptr(size_in), ptr(size_out), ptr(pos_map), ptr(out),
            out.stride(0), out.stride(1), _C.stream_ptr())
    return out


# ------------------------------------------------------------------------------------ GEMM
OUT_BF16, OUT_F32, OUT_F32_ACCUM = 0, 1, 2
ACT_NONE, ACT_RELU = 0, 1


def _epi(bias=None, act=ACT_NONE, rng=None, drop_layer=0, drop_site=0, keep_prob=1.0,
         drop_row_offset=0, gate=None, gate_scale=1.0, residual=None, alpha=1.0, beta=0.0,
         colsum=None, relu_bits=None, gate_bits=None, keep_bits=None):
    e = _C.Epilogue()
    e.colsum = ptr(colsum)
    e.relu_bits = ptr(relu_bits)
    e.gate_bits = ptr(gate_bits)
    e.keep_bits = ptr(keep_bits)
    e.bias = ptr(bias)
    e.act = act
    e.rng = ptr(rng)
    e.drop_layer, e.drop_site = drop_layer, drop_site
    e.keep_prob = keep_prob
    e.drop_row_offset = drop_row_offset
    e.gate = ptr(gate)
    e.ld_gate = gate.stride(0) if gate is not None else 0
    e.gate_scale = gate_scale
    e.residual = ptr(residual)
    e.ld_res = residual.stride(0) if residual is not None else 0
    e.res_dtype = _dtype_code(residual) if residual is not None else 1
    e.alpha, e.beta = alpha, beta
    return e


def auto_split_k(M: int, N: int, K: int) -> int:
    """Split of the reduction for launches with too few 128x128 tiles to fill 256 CUs (e.g. the
    T5 projections at M = B*32): fp32 slabs + a combine kernel that applies the epilogue."""
    tiles = -(-M // 128) * -(-N // 128)
    if tiles >= 192 or K < 512:
        return 1
    return int(max(1, min(-(-384 // tiles), K // 256, 8)))


def gemm(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
         out: torch.Tensor | None = None, out_mode: int = OUT_BF16, split_k: int | None = None,
         **epi):
    """2-D GEMM: op(a) (M x K) . op(b) (K x N). a/b bf16 with unit inner stride.
    trans_a: a is stored (K, M); trans_b: b is stored (N, K) (a weight W[N][K]).
    split_k None: auto_split_k."""
    _dev(a, b, out)
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("gemm operands must be bfloat16")
    if a.stride(-1) != 1 or b.stride(-1) != 1:
        raise ValueError("gemm operands need unit inner stride")
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[0], b.shape[1]) if trans_b else (b.shape[1], b.shape[0])
    if K != Kb:
        raise ValueError(f"gemm inner dims differ: {K} vs {Kb}")
    odt = torch.bfloat16 if out_mode == OUT_BF16 else torch.float32
    if out is None:
        out = (torch.zeros if out_mode == OUT_F32_ACCUM else torch.empty)(
            (M, N), dtype=odt, device=a.device)
    if out.dtype != odt or tuple(out.shape) != (M, N) or out.stride(-1) != 1:
        raise ValueError("bad gemm output tensor")
    for name, dts in (("gate", (torch.bfloat16,)), ("residual", (torch.bfloat16, torch.float32))):
        t = epi.get(name)
        if t is not None and (tuple(t.shape) != (M, N) or t.dtype not in dts or t.stride(-1) != 1):
            raise ValueError(f"gemm {name} must be {dts} (M, N) with unit inner stride")
    bias = epi.get("bias")
    if bias is not None and (bias.numel() != N or bias.dtype != torch.float32):
        raise ValueError("gemm bias must be fp32 [N]")
    if epi.get("keep_bits") is not None and (epi.get("relu_bits") is None or epi.get("rng") is not None):
        raise ValueError("gemm keep_bits replaces rng's dropout draws in a relu_bits launch")
    for name in ("relu_bits", "gate_bits", "keep_bits"):
        t = epi.get(name)
        if t is not None:
            if not gemm_bits_supported(M, N, K, trans_a, trans_b, out_mode, split_k):
                raise ValueError(f"gemm {name}: this launch shape has no 1-bit gate path")
            rows = -(-M // 256) * 256
            if t.dtype != torch.int32 or tuple(t.shape) != (rows, N // 32) or not t.is_contiguous():
                raise ValueError(f"gemm {name} must be contiguous int32 ({rows}, {N // 32})")
            split_k = 1
    cs = epi.get("colsum")
    if cs is not None:
        rows = gemm_colsum_rows(M, N, K, trans_a, trans_b, out_mode, 1 if split_k is None else split_k)
        if not rows or cs.dtype != torch.float32 or tuple(cs.shape) != (rows, N) or not cs.is_contiguous():
            raise ValueError(f"gemm colsum must be fp32 ({rows}, {N}) and this launch must support it")
        split_k = 1
    e = _epi(**epi)
    if split_k is None:
        split_k = auto_split_k(M, N, K)
    ws = None
    if split_k > 1:  # fp32 partial slabs, summed into `out` by the library's reduce kernel
        ws = torch.empty(split_k * M * N, dtype=torch.float32, device=a.device)
    _C.call("mmt_gemm", M, N, K, ptr(a), int(trans_a), a.stride(0), ptr(b), int(trans_b),
            b.stride(0), ptr(out), out_mode, out.stride(0), 1, 0, 0, 0, split_k,
            _C.ctypes.byref(e), ptr(ws), 0 if ws is None else ws.numel(), _C.stream_ptr())
    return out


def gemm_bits_supported(M: int, N: int, K: int, trans_a: bool = False, trans_b: bool = True,
                        out_mode: int = OUT_BF16, split_k: int | None = 1) -> bool:
    """Whether gemm(..., relu_bits= / gate_bits=) works for this launch (the 256-wide bf16 NT
    path, the same launches that can write epilogue column sums)."""
    return gemm_colsum_rows(M, N, K, trans_a, trans_b, out_mode, 1 if split_k is None else split_k) > 0


def gemm_dropout_keep_bits(rng: torch.Tensor, layer: int, site: int, M: int, N: int,
                           keep_prob: float, row_offset: int = 0, out: torch.Tensor | None = None):
    """The counter-RNG dropout keeps of an (M, N) gemm output in the relu_bits layout: pass as
    gemm(..., relu_bits=, keep_bits=, keep_prob=) without rng for outputs bit-identical to
    gemm(..., rng=, drop_layer=layer, drop_site=site, drop_row_offset=row_offset) — the draws run
    as their own kernel (e.g. on a side stream) instead of in the GEMM epilogue."""
    _dev(rng, out)
    rows = -(-M // 256) * 256
    if out is None:
        out = torch.empty((rows, N // 32), dtype=torch.int32, device=rng.device)
    if N % 256 or out.dtype != torch.int32 or tuple(out.shape) != (rows, N // 32) or not out.is_contiguous():
        raise ValueError(f"gemm_dropout_keep_bits: N % 256 == 0, out contiguous int32 ({rows}, {N // 32})")
    _C.call("mmt_gemm_dropout_keep_bits", ptr(rng), layer, site, M, N, keep_prob, row_offset, ptr(out),
            _C.stream_ptr())
    return out


def gemm_colsum_rows(M: int, N: int, K: int, trans_a: bool = False, trans_b: bool = True,
                     out_mode: int = OUT_BF16, split_k: int = 1) -> int:
    """Rows of the (rows, N) fp32 slab a gemm(..., colsum=slab) fills with the column sums of
    each 256-row panel of its bf16 output; 0 when that launch cannot (use colsum instead)."""
    return _C.call("mmt_gemm_colsum_rows", M, N, K, int(trans_a), int(trans_b), out_mode, split_k)


def quant_rows_fp8(x2d: torch.Tensor, out=None, scale=None):
    """bf16 (R, K) rows -> (e4m3 uint8 (R, K), fp32 scale (R,)): scale = amax / 448 per row."""
    _dev(x2d)
    if x2d.dtype != torch.bfloat16 or x2d.dim() != 2 or x2d.stride(1) != 1:
        raise ValueError("quant_rows_fp8 takes bf16 (rows, K) with unit inner stride")
    R, Kd = x2d.shape
    out = torch.empty((R, Kd), dtype=torch.uint8, device=x2d.device) if out is None else out
    scale = torch.empty(R, dtype=torch.float32, device=x2d.device) if scale is None else scale
    _C.call("mmt_quant_rows_fp8", ptr(x2d), x2d.stride(0), R, Kd, ptr(out), out.stride(0),
            ptr(scale), _C.stream_ptr())
    return out, scale


def gemm_fp8(aq: torch.Tensor, sa: torch.Tensor, bq: torch.Tensor, sb: torch.Tensor,
             out: torch.Tensor | None = None, out_mode: int = OUT_BF16, **epi):
    """(aq (M, K) e4m3 . bq (N, K)^T e4m3) * sa[m] * sb[n] with the GEMM epilogue."""
    _dev(aq, sa, bq, sb, out)
    if aq.dtype != torch.uint8 or bq.dtype != torch.uint8:
        raise TypeError("gemm_fp8 operands are e4m3 bytes (uint8)")
    M, Kd = aq.shape
    N, Kb = bq.shape
    if Kd != Kb or sa.numel() != M or sb.numel() != N:
        raise ValueError("gemm_fp8 shapes")
    if out_mode not in (OUT_BF16, OUT_F32):
        raise ValueError("gemm_fp8 writes bf16 or fp32")
    odt = torch.bfloat16 if out_mode == OUT_BF16 else torch.float32
    if out is None:
        out = torch.empty((M, N), dtype=odt, device=aq.device)
    for name, dts in (("gate", (torch.bfloat16,)), ("residual", (torch.bfloat16, torch.float32))):
        t = epi.get(name)
        if t is not None and (tuple(t.shape) != (M, N) or t.dtype not in dts or t.stride(-1) != 1):
            raise ValueError(f"gemm_fp8 {name} must be {dts} (M, N) with unit inner stride")
    e = _epi(**epi)
    _C.call("mmt_gemm_fp8", M, N, Kd, ptr(aq), aq.stride(0), ptr(sa), ptr(bq), bq.stride(0), ptr(sb),
            ptr(out), out_mode, out.stride(0), _C.ctypes.byref(e), _C.stream_ptr())
    return out


# ----------------------------------------------------------------------------- top-k pruning
def topk_gather(x: torch.Tensor, scores: torch.Tensor, tokenset_idx, tokenset_k):
    """x (B, L, D) fp32/bf16, scores (B, L) fp32; tokenset_idx [(start, num)], tokenset_k [k].
    Returns (out (B, sum k, D), idx (B, sum k) int32)."""
    _dev(x, scores)
    B, L, D = x.shape
    if scores.shape != (B, L) or scores.dtype != torch.float32 or scores.stride(1) != 1:
        raise ValueError("scores must be fp32 (B, L) with unit inner stride")
    n = len(tokenset_idx)
    if n != len(tokenset_k):
        raise ValueError("tokenset_idx and tokenset_k differ in length")
    starts = (_C.ctypes.c_int32 * n)(*[int(s) for s, _ in tokenset_idx])
    lens = (_C.ctypes.c_int32 * n)(*[int(m) for _, m in tokenset_idx])
    ks = (_C.ctypes.c_int32 * n)(*[int(k) for k in tokenset_k])
    K = int(sum(int(k) for k in tokenset_k))
    out = torch.empty((B, K, D), dtype=x.dtype, device=x.device)
    idx = torch.empty((B, K), dtype=torch.int32, device=x.device)
    _C.call("mmt_topk_gather", ptr(x), _dtype_code(x), B, L, D, x.stride(0), x.stride(1),
            ptr(scores), scores.stride(0), n, starts, lens, ks, ptr(out), out.stride(0),
            out.stride(1), ptr(idx), _C.stream_ptr())
    return out, idx


def prune_importance(wsum: torch.Tensor) -> torch.Tensor:
    """(B, H, L) post-dropout attention row sums -> (B, L) importance (mean over keys, heads)."""
    _dev(wsum)
    B, H, L = wsum.shape
    scores = torch.empty((B, L), dtype=torch.float32, device=wsum.device)
    _C.call("mmt_prune_importance", ptr(wsum), B, H, L, ptr(scores), _C.stream_ptr())
    return scores


def gather_rows(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """out[b, i] = x[b, idx[b, i]]: x (B, L, D) fp32/bf16, idx (B, K) int32."""
    _dev(x, idx)
    B, L, D = x.shape
    if idx.dtype != torch.int32 or idx.dim() != 2 or idx.shape[0] != B or not idx.is_contiguous():
        raise ValueError("idx must be contiguous int32 (B, K)")
    K = idx.shape[1]
    out = torch.empty((B, K, D), dtype=x.dtype, device=x.device)
    _C.call("mmt_gather_rows", ptr(x), _dtype_code(x), B, L, D, x.stride(0), x.stride(1), ptr(idx),
            K, ptr(out), out.stride(0), out.stride(1), _C.stream_ptr())
    return out


def topk_scatter_bwd(dout: torch.Tensor, idx: torch.Tensor, L: int):
    _dev(dout, idx)
    B, K, D = dout.shape
    dx = torch.empty((B, L, D), dtype=dout.dtype, device=dout.device)
    _C.call("mmt_topk_scatter_bwd", ptr(dout), _dtype_code(dout), B, K, D, dout.stride(0),
            dout.stride(1), ptr(idx), L, ptr(dx), dx.stride(0), dx.stride(1), _C.stream_ptr())
    return dx


# ------------------------------------------------------------------------------- attention
class SetTable:
    """Host-side token-set table of one layer: contiguous sets tiling [0, L) and, per query set,
    the bitmask of key sets it attends to (the blockwise mask of token_sequencer.py:94-183)."""

    CAUSAL = 1 << 31  # MMT_SET_CAUSAL: causal within the set (Text, token_sequencer.py:76-82)

    def __init__(self, starts, lens, vis, causal=None):
        n = len(starts)
        if n > 16:
            raise ValueError("at most 16 token sets")
        self.n = n
        self.starts = (_C.ctypes.c_int32 * max(n, 1))(*starts)
        self.lens = (_C.ctypes.c_int32 * max(n, 1))(*lens)
        causal = causal or [False] * n
        self.vis = (_C.ctypes.c_uint32 * max(n, 1))(*[(v & 0xFFFF) | (self.CAUSAL if c else 0)
                                                     for v, c in zip(vis, causal)])
        self.L = int(sum(lens))

    @staticmethod
    def none(L):
        return SetTable([0], [L], [1])


def dropout_bits(rng: torch.Tensor, layer: int, site: int, rows: int, cols: int, keep_prob: float,
                 out: torch.Tensor | None = None):
    """Keep bitmask words (rows, ceil(cols/32)) int32, bit j of word (r, w) = keep(r, 32w + j).
    For a square (attention) mask the result is (2, W, LP), LP = roundup(L, 64): [0] the query-word
    image (bit j of word (w, pos(k)) = keep(32w + j, k), read by the forward and dQ kernels),
    [1] the key-word image (bit j of word (w, pos(q)) = keep(q, 32w + j), read by dK/dV), with
    pos(8g + 4h + i) = 8g + 2i + h (csrc/attention.hip TileMasks: SGPR lane masks)."""
    words = (cols + 31) // 32
    square = rows == cols
    if out is None:
        shape = (2, words, (rows + 63) // 64 * 64) if square else (rows, words)
        out = torch.empty(shape, dtype=torch.int32, device=rng.device)
    out_t = ptr(out[1]) if square else None
    _C.call("mmt_dropout_bits", ptr(rng), layer, site, rows, cols, keep_prob,
            ptr(out[0] if square else out), out_t, _C.stream_ptr())
    return out


def _qkv_geo(qkv: torch.Tensor, H: int):
    if qkv.dim() != 3 or qkv.stride(2) != 1 or qkv.dtype != torch.bfloat16:
        raise ValueError("qkv must be bf16 (B, L, 3*H*Dh) with unit inner stride")
    B, L, three_d = qkv.shape
    if three_d % (3 * H):
        raise ValueError("qkv last dim must be 3*H*Dh")
    return B, L, three_d // (3 * H)


def _check_attn_bits(bits: torch.Tensor, L: int):
    want = (2, (L + 31) // 32, (L + 63) // 64 * 64)
    if tuple(bits.shape) != want or bits.dtype != torch.int32 or not bits.is_contiguous():
        raise ValueError(f"attention dropout needs the square mask of dropout_bits(.., L, L, ..): "
                         f"contiguous int32 {want}, got {tuple(bits.shape)}")


def attn_fwd_resident(L: int, Dh: int, bias: bool = False) -> bool:
    """Whether mmt_attn_fwd takes the K/V-resident kernel (attn_fwd_res_kernel: Dh 64,
    32 < L <= 320, no additive bias; MMT_ATTN_RES=0 disables it) — csrc/attention.hip."""
    import os
    return os.environ.get("MMT_ATTN_RES", "1") != "0" and Dh == 64 and not bias and 32 < L <= 320


def attn_bwd_resident(L: int, Dh: int) -> bool:
    """Whether mmt_attn_bwd takes the two-phase K/V-resident kernel (attn_bwd_res_kernel: Dh 64,
    32 < L <= 320; MMT_ATTN_RES_BWD=0 disables it) — csrc/attention.hip."""
    import os
    return os.environ.get("MMT_ATTN_RES_BWD", "1") != "0" and Dh == 64 and 32 < L <= 320


def attn_fwd(qkv: torch.Tensor, H: int, scale: float, table: SetTable | None = None,
             drop_bits: torch.Tensor | None = None, keep_prob: float = 1.0,
             bias: torch.Tensor | None = None, out: torch.Tensor | None = None,
             wsum: torch.Tensor | None = None):
    """wsum (optional fp32 (B, H, L)): receives the per-query sum of the post-dropout attention
    weights (the pruning importance, compressed_attention.py:302-306)."""
    _dev(qkv, drop_bits, bias, out, wsum)
    B, L, Dh = _qkv_geo(qkv, H)
    t = table or SetTable.none(L)
    if t.L != L:
        raise ValueError(f"set table covers {t.L} tokens, sequence has {L}")
    if bias is not None and (tuple(bias.shape) != (H, L, L) or bias.dtype != torch.float32 or not bias.is_contiguous()):
        raise ValueError("bias must be contiguous fp32 (H, L, L)")
    if out is None:
        out = torch.empty((B, L, H * Dh), dtype=torch.bfloat16, device=qkv.device)
    lse = torch.empty((B, H, L), dtype=torch.float32, device=qkv.device)
    if drop_bits is not None:
        _check_attn_bits(drop_bits, L)
        drop_bits = drop_bits[0]
    if wsum is not None and (tuple(wsum.shape) != (B, H, L) or wsum.dtype != torch.float32
                             or not wsum.is_contiguous()):
        raise ValueError("wsum must be contiguous fp32 (B, H, L)")
    _C.call("mmt_attn_fwd", ptr(qkv), qkv.stride(0), qkv.stride(1), B, L, H, Dh, scale, t.n,
            t.starts, t.lens, t.vis, ptr(drop_bits), keep_prob, ptr(bias), ptr(out), out.stride(0),
            out.stride(1), ptr(lse), ptr(wsum), _C.stream_ptr())
    return out, lse


def attn_lp(L: int) -> int:
    """Padded row length of the attention dropout words and backward workspace (roundup(L, 64))."""
    return (L + 63) & ~63


def attn_bwd(qkv, o, dout, lse, H: int, scale: float, table: SetTable | None = None,
             drop_bits=None, keep_prob: float = 1.0, dqkv: torch.Tensor | None = None,
             bias_grad: torch.Tensor | None = None):
    """bias_grad (fp32 [3*H*Dh], optional) += column sums of dqkv (the QKV bias gradient)."""
    _dev(qkv, o, dout, lse, drop_bits, dqkv, bias_grad)
    B, L, Dh = _qkv_geo(qkv, H)
    t = table or SetTable.none(L)
    if dout.stride(-1) != 1 or o.stride(-1) != 1:
        raise ValueError("o/dout need unit inner stride")
    if dqkv is None:
        dqkv = torch.empty_like(qkv)
    # workspace: rowsum(dO O) of the tiled kernels / the row constants of the resident one
    delta = torch.empty((B * H * 2 * attn_lp(L),), dtype=torch.float32, device=qkv.device)
    if drop_bits is not None:
        _check_attn_bits(drop_bits, L)
    bits, bits_t = (None, None) if drop_bits is None else (drop_bits[0], drop_bits[1])
    if bias_grad is not None and (bias_grad.dtype != torch.float32 or bias_grad.numel() != 3 * H * Dh
                                  or not bias_grad.is_contiguous()):
        raise ValueError("bias_grad must be contiguous fp32 [3*H*Dh]")
    _C.call("mmt_attn_bwd", ptr(qkv), qkv.stride(0), qkv.stride(1), B, L, H, Dh, scale, t.n,
            t.starts, t.lens, t.vis, ptr(bits), ptr(bits_t), keep_prob, ptr(o), o.stride(0), o.stride(1),
            ptr(dout), dout.stride(0), dout.stride(1), ptr(lse), ptr(delta), ptr(dqkv),
            dqkv.stride(0), dqkv.stride(1), ptr(bias_grad), _C.stream_ptr())
    return dqkv


# ------------------------------------------------------------------------ seq LayerNorm etc.
def seqnorm_fwd(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float,
                out: torch.Tensor | None = None):
    """x (B, L, D) bf16 or fp32 (the residual stream) -> y bf16, mean, rstd (B, D) fp32."""
    _dev(x, gamma, beta, out)
    B, L, D = x.shape
    if out is None:
        out = torch.empty((B, L, D), dtype=torch.bfloat16, device=x.device)
    mean = torch.empty((B, D), dtype=torch.float32, device=x.device)
    rstd = torch.empty((B, D), dtype=torch.float32, device=x.device)
    _C.call("mmt_seqnorm_fwd", ptr(x), _dtype_code(x), x.stride(0), x.stride(1), B, L, D,
            ptr(gamma), ptr(beta), eps, ptr(out), out.stride(0), out.stride(1), ptr(mean),
            ptr(rstd), _C.stream_ptr())
    return out, mean, rstd


def seqnorm_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, addend=None, out=None):
    """dx (dtype of x) = LN backward (+ addend, dtype of x); dy bf16 or fp32."""
    _dev(dy, x, mean, rstd, gamma, dgamma, dbeta, addend, out)
    B, L, D = x.shape
    if addend is not None and addend.dtype != x.dtype:
        raise TypeError("addend must have the residual (x) dtype")
    if out is None:
        out = torch.empty((B, L, D), dtype=x.dtype, device=x.device)
    a_sb, a_st = (addend.stride(0), addend.stride(1)) if addend is not None else (0, 0)
    _C.call("mmt_seqnorm_bwd", ptr(dy), _dtype_code(dy), dy.stride(0), dy.stride(1), ptr(x),
            _dtype_code(x), x.stride(0), x.stride(1), B, L, D, ptr(mean), ptr(rstd), ptr(gamma),
            ptr(addend), a_sb, a_st, ptr(out), out.stride(0), out.stride(1), ptr(dgamma),
            ptr(dbeta), _C.stream_ptr())
    return out


def colsum(x2d: torch.Tensor, out: torch.Tensor):
    _dev(x2d, out)
    M, N = x2d.shape
    _C.call("mmt_colsum", ptr(x2d), _dtype_code(x2d), x2d.stride(0), M, N, ptr(out), _C.stream_ptr())
    return out


def seqnorm_dropout_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, addend, rng, layer: int,
                        site: int, keep_prob: float, row_offset: int, colsum=None):
    """seqnorm_bwd (bf16 dy, fp32 x / addend) returning (dx fp32, z bf16), z = the previous
    block's dropout backward of dx (dropout_bwd semantics, colsum += its column sums)."""
    _dev(dy, x, mean, rstd, gamma, dgamma, dbeta, addend, rng, colsum)
    B, L, D = x.shape
    if x.dtype != torch.float32 or dy.dtype != torch.bfloat16 or (addend is not None and addend.dtype != torch.float32):
        raise TypeError("seqnorm_dropout_bwd takes bf16 dy and fp32 x / addend")
    dx = torch.empty((B, L, D), dtype=torch.float32, device=x.device)
    z = torch.empty((B, L, D), dtype=torch.bfloat16, device=x.device)
    a_sb, a_st = (addend.stride(0), addend.stride(1)) if addend is not None else (0, 0)
    _C.call("mmt_seqnorm_dropout_bwd", ptr(dy), dy.stride(0), dy.stride(1), ptr(x), x.stride(0),
            x.stride(1), B, L, D, ptr(mean), ptr(rstd), ptr(gamma), ptr(addend), a_sb, a_st, ptr(dx),
            dx.stride(0), dx.stride(1), ptr(dgamma), ptr(dbeta), ptr(rng), layer, site, keep_prob,
            row_offset, ptr(z), z.stride(0), z.stride(1), ptr(colsum), _C.stream_ptr())
    return dx, z


UNMERGE_MAX_L = 512          # csrc/norm.hip kUnmergeMax: unmerged rows per sample
UNMERGE_MAX_L2 = 96 * 1024 // (64 * 4)   # the merged (L2, 64-column) fp32 panel in <= 96 KB LDS


def ln_unmerge_ok(L: int, L2: int) -> bool:
    """The shapes mmt_ln_unmerge_dropout_bwd accepts (its C-side check, csrc/norm.hip): at most
    512 unmerged rows AND a merged panel of at most 384 rows; otherwise the caller takes the
    three-kernel path (seqnorm_bwd -> tome_merge_bwd -> dropout_bwd)."""
    return L <= UNMERGE_MAX_L and L2 <= UNMERGE_MAX_L2


def ln_unmerge_dropout_bwd(dy, x, mean, rstd, gamma, dgamma, dbeta, addend, tome, rng, layer: int,
                           site: int, keep_prob: float, row_offset: int, bias_grad=None):
    """seqnorm_bwd (merged layout: dy bf16, x / addend fp32) -> tome_merge_bwd -> dropout_bwd in one
    launch: returns (g_in fp32 (B, L, D), z bf16 (B, L, D)); dgamma / dbeta / bias_grad accumulated.
    tome = (set_start, t, r, pos_map, size_in, size_out)."""
    _dev(dy, x, mean, rstd, gamma, dgamma, dbeta, addend, rng, bias_grad)
    B, L2, D = x.shape
    s0, t, r, pos, size_in, size_out = tome
    L = L2 + r
    if x.dtype != torch.float32 or dy.dtype != torch.bfloat16 or (addend is not None and addend.dtype != torch.float32):
        raise TypeError("ln_unmerge_dropout_bwd takes bf16 dy and fp32 x / addend")
    g_in = torch.empty((B, L, D), dtype=torch.float32, device=x.device)
    z = torch.empty((B, L, D), dtype=torch.bfloat16, device=x.device)
    a_sb, a_st = (addend.stride(0), addend.stride(1)) if addend is not None else (0, 0)
    _C.call("mmt_ln_unmerge_dropout_bwd", ptr(dy), dy.stride(0), dy.stride(1), ptr(x), x.stride(0),
            x.stride(1), B, L2, D, ptr(mean), ptr(rstd), ptr(gamma), ptr(addend), a_sb, a_st,
            ptr(dgamma), ptr(dbeta), L, s0, t, r, ptr(size_in), ptr(size_out), ptr(pos), ptr(g_in),
            g_in.stride(0), g_in.stride(1), ptr(rng), layer, site, keep_prob, row_offset, ptr(z),
            z.stride(0), z.stride(1), ptr(bias_grad), _C.stream_ptr())
    return g_in, z


def dropout_bwd(dy2d: torch.Tensor, rng, layer: int, site: int, keep_prob: float,
                row_offset: int = 0, out: torch.Tensor | None = None, colsum_out=None):
    """dz (bf16) = dy * keep / keep_prob; rng None: plain cast. colsum_out += column sums."""
    _dev(dy2d, rng, out, colsum_out)
    M, N = dy2d.shape
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=dy2d.device)
    _C.call("mmt_dropout_bwd", ptr(dy2d), _dtype_code(dy2d), dy2d.stride(0), M, N, ptr(rng), layer,
            site, keep_prob, row_offset, ptr(out), out.stride(0), ptr(colsum_out), _C.stream_ptr())
    return out


# ------------------------------------------------------------------------------- image stem
IMG_F32, IMG_U8 = 0, 2


def patch_im2col(img: torch.Tensor, patch: int, kh: int, kw: int, stride: int, normalize: bool = True,
                 out: torch.Tensor | None = None):
    """img (B, I, H, H, C) fp32 or uint8 -> bf16 [B*I*NP*OH*OW][kh*kw*C]."""
    _dev(img, out)
    if img.dim() != 5 or img.shape[2] != img.shape[3] or not img.is_contiguous():
        raise ValueError("image must be contiguous (B, I, H, H, C) (square, image_tokenizer.py:49-50)")
    B, I, H, _, C = img.shape
    if H % patch:
        raise ValueError(f"image size {H} not divisible by patch {patch}")
    code = {torch.float32: IMG_F32, torch.uint8: IMG_U8}.get(img.dtype)
    if code is None:
        raise TypeError("image dtype must be float32 or uint8")
    oh, ow = (patch - kh) // stride + 1, (patch - kw) // stride + 1
    rows = B * I * (H // patch) ** 2 * oh * ow
    if out is None:
        out = torch.empty((rows, kh * kw * C), dtype=torch.bfloat16, device=img.device)
    _C.call("mmt_patch_im2col", ptr(img), code, B, I, H, C, patch, kh, kw, stride, int(normalize),
            ptr(out), _C.stream_ptr())
    return out


def _f32(t, what):
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise TypeError(f"{what} must be contiguous fp32")


def maxpool_patch(conv: torch.Tensor, win: int):
    """conv fp32 (npatch*win, C) -> pooled fp32 (npatch, C), first-max argmax uint8."""
    _f32(conv, "conv output")
    rows, C = conv.shape
    npatch = rows // win
    pooled = torch.empty((npatch, C), dtype=torch.float32, device=conv.device)
    arg = torch.empty((npatch, C), dtype=torch.uint8, device=conv.device)
    _C.call("mmt_maxpool_patch", ptr(conv), npatch, win, C, ptr(pooled), ptr(arg), _C.stream_ptr())
    return pooled, arg


def maxpool_patch_bwd(dpooled: torch.Tensor, arg: torch.Tensor, win: int, out=None):
    _f32(dpooled, "dpooled")
    npatch, C = dpooled.shape
    if out is None:
        out = torch.empty((npatch * win, C), dtype=torch.bfloat16, device=dpooled.device)
    _C.call("mmt_maxpool_patch_bwd", ptr(dpooled), ptr(arg), npatch, win, C, ptr(out), _C.stream_ptr())
    return out


def maxpool2d(x: torch.Tensor, npatch: int, OH: int, OW: int, KP: int):
    """x fp32 (npatch*OH*OW, C) -> pooled fp32 (npatch*PH*PW, C) (KP x KP, stride 1, VALID) and
    the window slot of the first maximum (uint8)."""
    _f32(x, "conv output")
    C = x.shape[-1]
    if x.numel() != npatch * OH * OW * C:
        raise ValueError("maxpool2d: x is not (npatch*OH*OW, C)")
    rows = npatch * (OH - KP + 1) * (OW - KP + 1)
    y = torch.empty((rows, C), dtype=torch.float32, device=x.device)
    arg = torch.empty((rows, C), dtype=torch.uint8, device=x.device)
    _C.call("mmt_maxpool2d", ptr(x), npatch, OH, OW, C, KP, ptr(y), ptr(arg), _C.stream_ptr())
    return y, arg


def maxpool2d_bwd(dy: torch.Tensor, arg: torch.Tensor, npatch: int, OH: int, OW: int, KP: int):
    """-> bf16 (npatch*OH*OW, C): the gradient routed to each window's first maximum."""
    _f32(dy, "dpooled")
    C = dy.shape[-1]
    G = torch.empty((npatch * OH * OW, C), dtype=torch.bfloat16, device=dy.device)
    _C.call("mmt_maxpool2d_bwd", ptr(dy), ptr(arg), npatch, OH, OW, C, KP, ptr(G), _C.stream_ptr())
    return G


def im2col_same(x: torch.Tensor, npatch: int, H: int, W: int, KS: int):
    """x bf16 (npatch*H*W, C) -> (npatch*H*W, KS*KS*C) bf16 columns of a SAME KS x KS conv."""
    _dev(x)
    C = x.shape[-1]
    if x.dtype != torch.bfloat16 or x.numel() != npatch * H * W * C or not x.is_contiguous():
        raise ValueError("im2col_same: x must be contiguous bf16 (npatch*H*W, C)")
    cols = torch.empty((npatch * H * W, KS * KS * C), dtype=torch.bfloat16, device=x.device)
    _C.call("mmt_im2col_same", ptr(x), npatch, H, W, C, KS, ptr(cols), _C.stream_ptr())
    return cols


def col2im_same(dcols: torch.Tensor, npatch: int, H: int, W: int, C: int, KS: int):
    _f32(dcols, "column gradient")
    dx = torch.empty((npatch * H * W, C), dtype=torch.float32, device=dcols.device)
    _C.call("mmt_col2im_same", ptr(dcols), npatch, H, W, C, KS, ptr(dx), _C.stream_ptr())
    return dx


def groupnorm_gelu_fwd(x: torch.Tensor, groups: int, gamma, beta, eps: float, out=None):
    """x (B, R, C) fp32 contiguous -> gelu(GroupNorm(x)) bf16."""
    _f32(x, "groupnorm input")
    B, R, C = x.shape
    if out is None:
        out = torch.empty((B, R, C), dtype=torch.bfloat16, device=x.device)
    mean = torch.empty((B, groups), dtype=torch.float32, device=x.device)
    rstd = torch.empty((B, groups), dtype=torch.float32, device=x.device)
    _C.call("mmt_groupnorm_gelu_fwd", ptr(x), B, R, C, groups, eps, ptr(gamma), ptr(beta), ptr(out),
            ptr(mean), ptr(rstd), _C.stream_ptr())
    return out, mean, rstd


def groupnorm_gelu_bwd(dy, x, groups, gamma, beta, mean, rstd, dgamma, dbeta, dx=None,
                       accumulate=False):
    """dy, x, dx fp32 (B, R, C); accumulate: dx += result."""
    _f32(dy, "dy")
    _f32(x, "x")
    B, R, C = x.shape
    if dx is None:
        dx = torch.empty_like(x)
    _C.call("mmt_groupnorm_gelu_bwd", ptr(dy), ptr(x), B, R, C, groups, ptr(gamma), ptr(beta),
            ptr(mean), ptr(rstd), ptr(dx), int(accumulate), ptr(dgamma), ptr(dbeta), _C.stream_ptr())
    return dx


def stem_conv_pool(images: torch.Tensor, w: torch.Tensor, bias: torch.Tensor):
    """images (B, I, H, H, 3) uint8, w (64, 432) bf16 [out][(ky, kx, c)], bias fp32 (64,) ->
    (pooled (B*I*NP, 64) fp32, argmax (B*I*NP, 64) uint8): 12x12 s2 conv of each normalised
    16x16 patch + bias, max over its 3x3 map (first maximum)."""
    _dev(images, w, bias)
    if images.dtype != torch.uint8 or images.dim() != 5 or images.shape[-1] != 3 or \
            images.shape[2] != images.shape[3] or images.shape[2] % 16 or not images.is_contiguous():
        raise ValueError("stem_conv_pool takes contiguous uint8 (B, I, H, H, 3) images, H % 16 == 0")
    if w.dtype != torch.bfloat16 or tuple(w.shape) != (64, 432) or not w.is_contiguous():
        raise ValueError("stem_conv_pool weight must be contiguous bf16 (64, 432)")
    if bias.dtype != torch.float32 or bias.numel() != 64:
        raise ValueError("stem_conv_pool bias must be fp32 (64,)")
    B, I, H = images.shape[:3]
    n = B * I * (H // 16) ** 2
    pooled = torch.empty((n, 64), dtype=torch.float32, device=images.device)
    arg = torch.empty((n, 64), dtype=torch.uint8, device=images.device)
    _C.call("mmt_stem_conv_pool", ptr(images), B, I, H, ptr(w), ptr(bias), ptr(pooled), ptr(arg),
            _C.stream_ptr())
    return pooled, arg


def stem_conv_wgrad(images: torch.Tensor, dpooled: torch.Tensor, arg: torch.Tensor,
                    wgrad: torch.Tensor):
    """wgrad (64, 432) fp32 += the stem conv weight gradient from the pooled gradient (fp32
    (B*I*NP, 64)) and the forward's argmax, straight from the uint8 images (no im2col)."""
    _dev(images, dpooled, arg, wgrad)
    B, I, H = images.shape[:3]
    n = B * I * (H // 16) ** 2
    if tuple(dpooled.shape) != (n, 64) or dpooled.dtype != torch.float32 or not dpooled.is_contiguous():
        raise ValueError("dpooled must be contiguous fp32 (B*I*NP, 64)")
    if tuple(arg.shape) != (n, 64) or arg.dtype != torch.uint8 or not arg.is_contiguous():
        raise ValueError("argmax must be contiguous uint8 (B*I*NP, 64)")
    if tuple(wgrad.shape) != (64, 432) or wgrad.dtype != torch.float32 or not wgrad.is_contiguous():
        raise ValueError("wgrad must be contiguous fp32 (64, 432)")
    rows = _C.call("mmt_stem_conv_wgrad_slabs", B, I, H)
    slab = torch.empty((rows, 64 * 432), dtype=torch.float32, device=images.device)
    _C.call("mmt_stem_conv_wgrad", ptr(images), B, I, H, ptr(dpooled), ptr(arg), ptr(slab),
            slab.numel(), _C.stream_ptr())
    colsum(slab, wgrad.view(-1))
    return wgrad


def patch_positions(B: int, I: int, H: int, patch: int, Q: int, train: bool, rng=None, site: int = 0,
                    sample_offset: int = 0, device=None):
    npatch = (H // patch) ** 2
    dev = device if device is not None else rng.device
    rt = torch.empty((B, I * npatch), dtype=torch.int32, device=dev)
    ct = torch.empty((B, I * npatch), dtype=torch.int32, device=dev)
    _C.call("mmt_patch_positions", ptr(rng), site, B, I, H, patch, Q, int(train), sample_offset,
            ptr(rt), ptr(ct), _C.stream_ptr())
    return rt, ct


# ---------------------------------------------------------------------------------- glue
def rmsnorm(x2d: torch.Tensor, w: torch.Tensor, eps: float, out=None):
    rows, D = x2d.shape
    if out is None:
        out = torch.empty_like(x2d)
    _C.call("mmt_rmsnorm_fwd", ptr(x2d), rows, D, ptr(w), eps, ptr(out), _C.stream_ptr())
    return out


def embedding_gather(ids: torch.Tensor, table: torch.Tensor, out=None):
    n = ids.numel()
    vocab, D = table.shape
    if out is None:
        out = torch.empty((n, D), dtype=table.dtype, device=table.device)
    _C.call("mmt_embedding_gather", ptr(ids), n, D, ptr(table), vocab, ptr(out), _C.stream_ptr())
    return out


def cast_f32_bf16(a: torch.Tensor, out: torch.Tensor):
    _C.call("mmt_cast_f32_bf16", ptr(a), ptr(out), a.numel(), _C.stream_ptr())
    return out
