"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

Two CPU restatements of the reference's ToMe (multi_modal_transformers/tokenizers/
token_compression.py):

* ``literal_*``: numpy, op for op as the reference writes it (norm, matmul, max/argmax,
  ``argsort(...)[:, ::-1]``, r sequential scatter-adds, ``merge_wavg``). numpy's reduction order is
  not the kernel's, so values can differ in the last ulp; it pins the *semantics* (index
  conventions, concat order, tie rules) and the hand-derived KATs of SURVEY.md §8c.
* ``canon_*``: ctypes wrappers around oracle/tome_ref.c, the canonical-arithmetic restatement the
  HIP kernels must match bit for bit.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None


# ----------------------------------------------------------------------------- literal numpy
def literal_bipartite_soft_matching(metric: np.ndarray, r: int, class_token=False,
                                    distill_token=False):
    """token_compression.py:54-112. Returns (merge_fn, unm_idx, src_idx, dst_idx) or None for
    the r <= 0 do-nothing branch (:69-70)."""
    protected = int(class_token) + int(distill_token)
    t = metric.shape[1]
    r = min(r, (t - protected) // 2)
    if r <= 0:
        return None
    metric = metric.astype(np.float32)
    metric = metric / np.linalg.norm(metric, axis=-1, keepdims=True)
    a, b = metric[..., ::2, :], metric[..., 1::2, :]
    scores = np.matmul(a, np.swapaxes(b, -1, -2))
    if class_token:
        scores[..., 0, :] = -np.inf
    if distill_token:
        scores[..., :, 0] = -np.inf
    node_max = scores.max(axis=-1)
    node_idx = scores.argmax(axis=-1)
    edge_idx = np.argsort(node_max, axis=-1, kind="stable")[:, ::-1][..., None]
    unm_idx = edge_idx[..., r:, :]
    src_idx = edge_idx[..., :r, :]
    dst_idx = np.take_along_axis(node_idx[..., None], src_idx, axis=-2)

    def merge(x: np.ndarray, mode="sum") -> np.ndarray:
        n = x.shape[0]
        unm = np.take_along_axis(x[..., ::2, :], unm_idx, axis=1)
        src = np.take_along_axis(x[..., ::2, :], src_idx, axis=1)
        dst = np.array(x[..., 1::2, :])
        if mode == "sum":
            for i in range(dst_idx.shape[1]):
                dst[np.arange(n), dst_idx[:, i, 0], :] += src[:, i, :]
        if distill_token:
            return np.concatenate([unm[:, :1], dst[:, :1], unm[:, 1:], dst[:, 1:]], axis=1)
        return np.concatenate([unm, dst], axis=1)

    return merge, unm_idx[..., 0].astype(np.int32), src_idx[..., 0].astype(np.int32), \
        dst_idx[..., 0].astype(np.int32)


def literal_merge_wavg(merge, x: np.ndarray, size: np.ndarray | None = None):
    """token_compression.py:114-129."""
    if size is None:
        size = np.ones_like(x[..., 0, None])
    x = merge(x * size, mode="sum")
    size = merge(size, mode="sum")
    return x / size, size


# ----------------------------------------------------------------------------- canonical C
def _lib():
    global _LIB
    if _LIB is None:
        so = _HERE / "liboracle.so"
        src = _HERE / "tome_ref.c"
        if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
            subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
        lib = ctypes.CDLL(str(so))
        P = ctypes.c_void_p
        I = ctypes.c_int
        L = ctypes.c_int64
        lib.tome_ref_match.argtypes = [P, I, I, I, I, L, L, L, I, I, P, P, P, P]
        lib.tome_ref_match.restype = I
        lib.tome_ref_merge_wavg.argtypes = [P, P, I, I, I, I, I, P, P, P, P, P]
        lib.tome_ref_merge_wavg.restype = I
        _LIB = lib
    return _LIB


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def canon_match(metric: np.ndarray, r: int, flags: int = 0):
    """metric: (n, t, c) or (n, t, heads, c) fp32 (bf16 inputs must be widened exactly first).
    Returns (unm, src, dst, node_max) with r already clamped by the caller."""
    m = np.ascontiguousarray(metric, dtype=np.float32)
    if m.ndim == 3:
        m = m[:, :, None, :]
    n, t, h, c = m.shape
    ta = (t + 1) // 2
    unm = np.empty((n, ta - r), np.int32)
    src = np.empty((n, r), np.int32)
    dst = np.empty((n, r), np.int32)
    nmax = np.empty((n, ta), np.float32)
    rc = _lib().tome_ref_match(_ptr(m), n, t, h, c, t * h * c, h * c, c, r, flags, _ptr(unm),
                               _ptr(src), _ptr(dst), _ptr(nmax))
    assert rc == 0
    return unm, src, dst, nmax


def canon_merge_wavg(x: np.ndarray, size: np.ndarray | None, unm, src, dst, r: int,
                     flags: int = 0):
    """x: (n, t, D) fp32 token set; size: (n, t) fp32 or None. Returns (x_out, size_out)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, t, D = x.shape
    s = None if size is None else np.ascontiguousarray(size, dtype=np.float32)
    xo = np.empty((n, t - r, D), np.float32)
    so = np.empty((n, t - r), np.float32)
    rc = _lib().tome_ref_merge_wavg(_ptr(x), _ptr(s), n, t, D, r, flags,
                                    _ptr(np.ascontiguousarray(unm, np.int32)),
                                    _ptr(np.ascontiguousarray(src, np.int32)),
                                    _ptr(np.ascontiguousarray(dst, np.int32)), _ptr(xo), _ptr(so))
    assert rc == 0
    return xo, so


def canon_pos_map(unm, src, dst, t: int, r: int, flags: int = 0) -> np.ndarray:
    """For each set token, the merged row it lands in (used by the merge backward)."""
    n = unm.shape[0]
    ta = (t + 1) // 2
    nu = ta - r
    dis = bool(flags & 2)
    pos = np.full((n, t), -1, np.int32)
    for b in range(n):
        def row_of_dst(j):
            return (1 if j == 0 else nu + j) if dis else nu + j

        def row_of_unm(u):
            return (0 if u == 0 else u + 1) if dis else u

        for u in range(nu):
            pos[b, 2 * unm[b, u]] = row_of_unm(u)
        for j in range(t // 2):
            pos[b, 2 * j + 1] = row_of_dst(j)
        for i in range(r):
            pos[b, 2 * src[b, i]] = row_of_dst(dst[b, i])
    return pos


def canon_merge_bwd(g_out: np.ndarray, size_in, size_out, pos_map) -> np.ndarray:
    """d x_in = g_out[pos] * size_in / size_out[pos]  (fp32)."""
    n, t = pos_map.shape
    s = np.ones((n, t), np.float32) if size_in is None else size_in.astype(np.float32)
    g = np.take_along_axis(g_out, pos_map[..., None].astype(np.int64), axis=1)
    S = np.take_along_axis(size_out, pos_map.astype(np.int64), axis=1)
    return ((g * s[..., None]) / S[..., None]).astype(np.float32)


def topk_tokens(embeddings: np.ndarray, scores: np.ndarray, tokenset_idx, tokenset_k):
    """Literal restatement of token_compression.py:15-46 for one sample: jax.lax.top_k per set
    (descending; equal values keep the lower index first; lax's float total order, NaN largest),
    indices + set start, concatenated, then take(embeddings, ids, axis=0)."""
    def key(v):
        v = np.float32(v)
        if np.isnan(v):
            return (1, 0)
        return (0, float(v) if v != 0 else (0.0 if not np.signbit(v) else -0.0),
                0 if np.signbit(v) else 1)
    ids = []
    for (start, num), k in zip(tokenset_idx, tokenset_k):
        sub = scores[start:start + num]
        order = sorted(range(num), key=lambda i: (tuple(-x for x in key(sub[i])), i))
        ids.extend(start + i for i in order[:k])
    ids = np.asarray(ids, dtype=np.int32)
    return embeddings[ids], ids
