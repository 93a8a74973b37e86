"""Flat parameter storage for the training path.

Every trainable tensor is a view into ONE fp32 master buffer, with parallel flat buffers for its
bf16 shadow (what the MFMA GEMMs read), its fp32 gradient (what the backward kernels accumulate
into, zeroed by one memset per step) and the AdamW moments. Consequences on MI355X:
  * the optimizer is one fused kernel launch over the whole model (mmt_adamw);
  * the data-parallel gradient all-reduce runs on a few large contiguous buckets (RCCL over
    xGMI) instead of hundreds of small tensors;
  * no per-parameter allocation or autograd accumulation kernels exist on the hot path.
Views are 64-element aligned (256 B) so every GEMM operand base is 16-B aligned.

Frozen parameters (the T5 encoder, t5_base.py:14 stop_gradient) live in a separate bf16-only
store: they have no master copy, no gradient and no optimizer state.

Initialisers restate the Flax ones the reference's YAML names (he_normal = variance_scaling(2,
fan_in, truncated_normal), normal(0.01) biases, LayerNorm ones/zeros, ...).
"""
from __future__ import annotations

import math
import weakref
from dataclasses import dataclass
from typing import Callable, Dict, List, Tuple

import torch

ALIGN = 64


def _fans(shape, in_axis=-2, out_axis=-1):
    """flax.linen.initializers._compute_fans for a Flax-layout shape (..., in, out)."""
    if len(shape) < 2:
        return shape[0], shape[0]
    rf = 1
    for i, s in enumerate(shape):
        if i not in (len(shape) + in_axis, len(shape) + out_axis):
            rf *= s
    return shape[in_axis] * rf, shape[out_axis] * rf


def he_normal(flax_shape):
    """variance_scaling(2.0, 'fan_in', 'truncated_normal') on the Flax kernel shape."""
    fan_in, _ = _fans(flax_shape)
    std = math.sqrt(2.0 / fan_in) / 0.87962566103423978

    def init(t: torch.Tensor, g: torch.Generator):
        with torch.no_grad():
            t.copy_(torch.fmod(torch.randn(t.shape, generator=g), 2.0) * std)  # approx trunc at 2 sd
        return t
    return init


def normal(std):
    def init(t, g):
        with torch.no_grad():
            t.copy_(torch.randn(t.shape, generator=g) * std)
        return t
    return init


def variance_scaling_normal(scale, flax_shape):
    fan_in, _ = _fans(flax_shape)
    return normal(math.sqrt(scale / fan_in))


def const(v):
    def init(t, g):
        with torch.no_grad():
            t.fill_(v)
        return t
    return init


@dataclass
class Param:
    name: str
    shape: Tuple[int, ...]
    init: Callable
    offset: int = -1
    data: torch.Tensor | None = None      # fp32 master view
    bf16: torch.Tensor | None = None      # bf16 shadow view
    transposed: bool = False              # also keep a transposed bf16 shadow (2-D weights)
    bf16_t: torch.Tensor | None = None    # its (cols, rows) view
    fp8: bool = False                     # also keep an e4m3 shadow with one scale per row
    q8: torch.Tensor | None = None        # (rows, cols) uint8 e4m3 view
    q8_scale: torch.Tensor | None = None  # (rows,) fp32
    grad: torch.Tensor | None = None      # fp32 grad view

    @property
    def numel(self):
        return math.prod(self.shape)


class ParamStore:
    def __init__(self):
        self.params: List[Param] = []
        self.by_name: Dict[str, Param] = {}
        self.n = 0
        self.flat = self.flat_bf16 = self.flat_grad = self.m = self.v = None

    def add(self, name: str, shape, init, transposed: bool = False, fp8: bool = False) -> Param:
        if name in self.by_name:
            raise KeyError(f"duplicate parameter {name}")
        if (transposed or fp8) and len(shape) != 2:
            raise ValueError("only 2-D parameters keep transposed / fp8 shadows")
        p = Param(name, tuple(int(s) for s in shape), init, transposed=transposed, fp8=fp8)
        p.offset = self.n
        self.n += (p.numel + ALIGN - 1) // ALIGN * ALIGN
        self.params.append(p)
        self.by_name[name] = p
        return p

    def materialize(self, device, seed: int = 0):
        """Allocate the flat buffers, initialise every parameter deterministically on the host
        (torch.Generator(seed), in declaration order) and upload once."""
        g = torch.Generator().manual_seed(seed)
        host = torch.zeros(self.n, dtype=torch.float32)
        for p in self.params:
            view = host[p.offset:p.offset + p.numel].view(p.shape)
            p.init(view, g)
        self.flat = host.to(device)
        self.flat_bf16 = self.flat.to(torch.bfloat16)
        self.flat_grad = torch.zeros_like(self.flat)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        # transposed bf16 shadows of the 2-D weights (same offsets, (cols, rows) views): every
        # dX = dY . W then runs as an NT GEMM; refreshed after each optimizer step
        tps = [p for p in self.params if p.transposed]
        self.flat_bf16_t = torch.zeros_like(self.flat_bf16) if tps else None
        self._t_desc, self._t_tiles = None, 0
        # e4m3 shadows (+ one fp32 scale per row) of the fp8-path weights, same offsets
        f8 = [p for p in self.params if p.fp8]
        self.flat_fp8 = torch.zeros(self.n, dtype=torch.uint8, device=device) if f8 else None
        n_rows = sum((p.shape[0] + 3) // 4 * 4 for p in f8)
        self.fp8_scale = torch.ones(max(n_rows, 1), dtype=torch.float32, device=device) if f8 else None
        if tps:
            rows = []
            tiles = 0
            for p in tps:
                r, c = p.shape
                rows += [p.offset, p.offset, r, c, tiles]
                tiles += -(-r // 64) * -(-c // 64)
            self._t_desc = torch.tensor(rows, dtype=torch.int64, device=device)
            self._t_tiles = tiles
        self._bind()
        self.refresh_transposed()
        self.refresh_fp8()
        return self

    def refresh_fp8(self):
        """Re-quantise the e4m3 weight shadows from the bf16 shadow (one launch per weight,
        captured into the step graph after AdamW)."""
        if self.flat_fp8 is None:
            return
        if not self.flat_bf16.is_cuda:
            raise RuntimeError("fp8 shadows live on the device")
        from . import _kernels as K
        for p in self.params:
            if p.fp8:
                K.quant_rows_fp8(p.bf16, out=p.q8, scale=p.q8_scale)

    def refresh_transposed(self):
        """Re-derive the transposed bf16 shadows from the bf16 shadow (one batched launch; on a
        host-resident store, used by the checkpoint tools, a host transpose)."""
        if self.flat_bf16_t is None:
            return
        if self.flat_bf16.is_cuda:
            from . import _C
            _C.call("mmt_transpose_bf16_batched", _C.ptr(self.flat_bf16), _C.ptr(self.flat_bf16_t),
                    _C.ptr(self._t_desc), self._t_desc.numel() // 5, self._t_tiles, _C.stream_ptr())
        else:
            for p in self.params:
                if p.transposed:
                    p.bf16_t.copy_(p.bf16.t())

    def _bind(self):
        for p in self.params:
            sl = slice(p.offset, p.offset + p.numel)
            p.data = self.flat[sl].view(p.shape)
            p.bf16 = self.flat_bf16[sl].view(p.shape)
            p.grad = self.flat_grad[sl].view(p.shape)
            if p.transposed:
                p.bf16_t = self.flat_bf16_t[sl].view(p.shape[1], p.shape[0])
        so = 0
        for p in self.params:
            if p.fp8:
                p.q8 = self.flat_fp8[p.offset:p.offset + p.numel].view(p.shape)
                p.q8_scale = self.fp8_scale[so:so + p.shape[0]]
                so += (p.shape[0] + 3) // 4 * 4

    def zero_grad(self):
        self.flat_grad.zero_()

    # ------------------------------------------------------------------ deterministic mode
    det_fx = None  # int64 fixed-point shadow of flat_grad while the mode is on

    def set_deterministic(self, on: bool = True):
        """Deterministic mode (include/mmt_api.h mmt_set_deterministic): the gradient sums that
        are fp32 atomics otherwise go to an int64 fixed-point shadow of flat_grad (integer adds:
        order-independent), added into flat_grad by det_flush. Resolution 2^-36 per
        contribution, range |sum| < 2^27 per element; a NaN / Inf or |v| >= 2^15 contribution
        bypasses the shadow as a plain fp32 atomic, so it still shows in the gradient (and at
        most 4096 shadow contributions per element per flush cannot wrap the int64).
        The library keeps ONE registration per process: a second store asking for it while
        another LIVE store holds it raises (its gradient sites would otherwise silently take the
        registration from the first). The registration refers to its store weakly: a store
        dropped without close() counts as released, and the next store to ask takes the
        registration over. Until then the class keeps the two device buffers the library points
        at (flat_grad and the shadow) alive, so no kernel can write into freed memory; the
        takeover (or set_deterministic(False) / close() / ``with store.deterministic():``) lets
        them go. Synchronous, so call outside graph capture."""
        from . import _C
        if on:
            owner = ParamStore._det_owner() if ParamStore._det_owner is not None else None
            if owner is not None and owner is not self:
                raise RuntimeError("deterministic mode is registered by another ParamStore; "
                                   "call its set_deterministic(False) / close() first")
            if self.det_fx is None:
                self.det_fx = torch.zeros(self.n, dtype=torch.int64, device=self.flat_grad.device)
            _C.call("mmt_set_deterministic", _C.ptr(self.flat_grad), _C.ptr(self.det_fx), self.n)
            ParamStore._det_owner = weakref.ref(self)
            ParamStore._det_buffers = (self.flat_grad, self.det_fx)
        else:
            if self._holds_det():
                _C.call("mmt_set_deterministic", None, None, 0)
                ParamStore._det_owner = None
                ParamStore._det_buffers = None
            self.det_fx = None

    _det_owner = None    # weakref.ref to the registered store
    _det_buffers = None  # (flat_grad, shadow) the library points at while registered

    def _holds_det(self) -> bool:
        return ParamStore._det_owner is not None and ParamStore._det_owner() is self

    def close(self):
        """Release the deterministic-mode registration if this store holds it (the explicit
        form of leaving the mode; nothing touches the device from __del__)."""
        self.set_deterministic(False)

    def deterministic(self):
        """``with store.deterministic(): ...`` — the mode on for the block, released on exit."""
        import contextlib

        @contextlib.contextmanager
        def _cm():
            self.set_deterministic(True)
            try:
                yield self
            finally:
                self.set_deterministic(False)
        return _cm()

    def det_flush(self, lo: int = 0, hi: int | None = None):
        """flat_grad[lo:hi] += shadow * 2^-36, shadow[lo:hi] = 0 (no-op outside the mode)."""
        if self.det_fx is None:
            return
        from . import _C
        hi = self.n if hi is None else hi
        _C.call("mmt_det_flush", _C.ptr(self.flat_grad[lo:]), _C.ptr(self.det_fx[lo:]), hi - lo,
                _C.stream_ptr())

    def sync_shadow(self):
        """Re-derive the bf16 shadow after the master was modified outside AdamW."""
        self.flat_bf16.copy_(self.flat.to(torch.bfloat16))
        self.refresh_transposed()
        self.refresh_fp8()

    def num_params(self) -> int:
        return sum(p.numel for p in self.params)

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {p.name: p.data for p in self.params}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]):
        for p in self.params:
            p.data.copy_(sd[p.name].to(p.data.device, torch.float32).view(p.shape))
        self.sync_shadow()


class FrozenStore:
    """bf16-only parameters (no grad, no optimizer state)."""

    def __init__(self):
        self.params: List[Param] = []
        self.by_name: Dict[str, Param] = {}
        self.n = 0
        self.flat_bf16 = None

    def add(self, name, shape, init) -> Param:
        p = Param(name, tuple(int(s) for s in shape), init)
        p.offset = self.n
        self.n += (p.numel + ALIGN - 1) // ALIGN * ALIGN
        self.params.append(p)
        self.by_name[name] = p
        return p

    def materialize(self, device, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        host = torch.zeros(self.n, dtype=torch.float32)
        for p in self.params:
            p.init(host[p.offset:p.offset + p.numel].view(p.shape), g)
        self.flat_bf16 = host.to(torch.bfloat16).to(device)
        for p in self.params:
            p.bf16 = self.flat_bf16[p.offset:p.offset + p.numel].view(p.shape)
        return self

    def num_params(self) -> int:
        return sum(p.numel for p in self.params)
