"""Dense and sequence-LayerNorm building blocks with explicit forward / backward on libmmt_hip.

The training step is an explicit forward + reverse schedule of C-ABI kernels (no torch autograd
tape, no per-op Python allocation of gradients): each layer object declares its parameters in
the flat ParamStore, ``fwd`` returns activations plus what its ``bwd`` needs, and ``bwd`` writes
parameter gradients straight into the flat gradient buffer (split-K fp32 atomics for dW, column
sums for biases) and returns the input gradient.
"""
from __future__ import annotations

import math
import os

import torch

from . import _kernels as K
from .params import ParamStore, const, he_normal, normal

DROP_ATTN, DROP_ATTN_OUT, DROP_MLP_HIDDEN, DROP_MLP_OUT = 0, 1, 2, 3  # dropout "sites" per layer


class wgrad_overlap:
    """Within this context every Dense.bwd issues its weight-gradient GEMM (and bias column sum)
    on a second HIP stream, forked from the main stream at the call, so the MFMA-bound dW
    products run beside the latency- and memory-bound kernels of the backward's critical path
    (attention backward, LayerNorm backward, ToMe unmerge). The operands stay referenced until
    the join on exit (main waits for the stream), so the allocator cannot hand their memory to
    the main stream early; the join also precedes any all-reduce of the gradients. Works the
    same under HIP-graph capture (fork / join by events)."""
    _streams: dict = {}
    active = None  # (stream, keep-alive list)

    def __init__(self, device):
        key = torch.device(device).index
        if key not in wgrad_overlap._streams:
            wgrad_overlap._streams[key] = torch.cuda.Stream(device=device)
        self.stream = wgrad_overlap._streams[key]

    enabled = os.environ.get("MMT_WGRAD_OVERLAP", "1") != "0"  # benchmarking knob

    def __enter__(self):
        if wgrad_overlap.enabled:
            wgrad_overlap.active = (self.stream, [])
        return self

    # blocks the dW stream may run behind before the main stream waits for it; 0 = no per-block
    # join, every dW joins at the end of the backward (or its DDP stage). Round 3 (B = 512, 2
    # interleaved rounds): 0 14.92k, 1 14.72k, 2 14.74k, 3 14.77k samples/s — with the round-3
    # kernels the side queue keeps up without the join
    lag = int(os.environ.get("MMT_WGRAD_LAG", "0"))
    _marks: list = []
    @staticmethod
    def block_done():
        """End of one block's backward: with lag > 0 the main stream waits for the dW work of the
        block `lag` blocks back (round 2: without it the graph ran the whole backward's critical
        path first and the side stream's dW products late — the side queue idle for the first
        6 ms, then 2.5 ms of dW alone; round 3's faster kernels reversed the balance: lag 0, the
        default, is 1.4 % faster)."""
        a = wgrad_overlap.active
        if a is None or wgrad_overlap.lag <= 0:
            return
        ev = torch.cuda.Event()
        ev.record(a[0])
        wgrad_overlap._marks.append(ev)
        if len(wgrad_overlap._marks) > wgrad_overlap.lag:
            torch.cuda.current_stream().wait_event(wgrad_overlap._marks.pop(0))

    def __exit__(self, *exc):
        wgrad_overlap._marks.clear()
        if wgrad_overlap.active is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
            wgrad_overlap.active[1].clear()
            wgrad_overlap.active = None
        return False


_TN_BM = 256 if os.environ.get("MMT_TN_BM") == "256" else 384  # as csrc/gemm.hip's tile choice
# workgroups a weight-gradient launch in the step is split for (MMT_WGRAD_WGS overrides): the
# split-K slab bytes written and combined scale with it, the launch's CU-time does not, and the
# launches share the chip with the main queue's backward anyway — half the chip measured +0.8-1 %
# per step over a full-chip split (15,451 / 15,501 vs 15,326 / 15,338 samples/s; 64: -6 %)
_WGRAD_WGS = int(os.environ.get("MMT_WGRAD_WGS", "128"))


def split_k_for(n_out: int, k_out: int, m_red: int, wgs: int = 0) -> int:
    """Split of the M-reduction of a weight-gradient GEMM so the launch runs ~wgs workgroups
    (default _WGRAD_WGS = 128, half the chip: the dW launches run on the side queue beside the
    main queue's backward; 256 fills the chip once, as the standalone bench probe does): the TN
    products run on the direct-to-LDS kernel at one workgroup per CU (csrc/gemm.hip
    gemm_tn_dma_kernel: 384 x 192 tiles where n_out % 384 == 0, else 256 x 192), so the split is
    sized in ITS tiles."""
    bm = _TN_BM if n_out % 384 == 0 else 256
    tiles = math.ceil(n_out / bm) * math.ceil(k_out / 192)
    want = max(1, (wgs or _WGRAD_WGS) // tiles)
    return int(max(1, min(want, m_red // 256, 128)))


class Dense:
    """flax.linen.Dense (kernel (in, out) in Flax; stored here as W[out][in] so the forward is
    the NT GEMM y = x W^T and the GEMM reads both operands along the reduction)."""

    def __init__(self, store: ParamStore, name: str, in_f: int, out_f: int, use_bias: bool = True,
                 kernel_init=None, bias_init=None, fp8: bool = False):
        self.in_f, self.out_f = in_f, out_f
        # fp8: the forward product runs in e4m3 (per-row activation scales, per-output-channel
        # weight scales, csrc/gemm.hip gemm_fp8_nt_kernel); the backward stays bf16 (straight-through)
        self.fp8 = fp8
        self.w = store.add(f"{name}/kernel", (out_f, in_f), kernel_init or he_normal((in_f, out_f)),
                           transposed=True, fp8=fp8)
        self.b = store.add(f"{name}/bias", (out_f,), bias_init or normal(0.01)) if use_bias else None

    def fwd(self, x2d: torch.Tensor, out=None, out_mode=K.OUT_BF16, **epi) -> torch.Tensor:
        if self.fp8:
            xq, sx = K.quant_rows_fp8(x2d)
            return K.gemm_fp8(xq, sx, self.w.q8, self.w.q8_scale, out=out, out_mode=out_mode,
                              bias=self.b.data if self.b else None, **epi)
        return K.gemm(x2d, self.w.bf16, trans_b=True, bias=self.b.data if self.b else None,
                      out=out, out_mode=out_mode, **epi)

    def bwd(self, dy2d: torch.Tensor, x2d: torch.Tensor, need_dx: bool = True,
            bias_grad_done: bool = False, dx_out=None, dy_colsum=None, **dx_epi):
        """dy_colsum: the (panels, out) slab of per-256-row column sums of dy that the GEMM
        producing dy wrote in its epilogue (gemm colsum=); the bias gradient then sums the slab
        instead of re-reading dy."""
        M = dy2d.shape[0]

        def wgrad():
            K.gemm(dy2d, x2d, trans_a=True, out=self.w.grad, out_mode=K.OUT_F32_ACCUM,
                   split_k=split_k_for(self.out_f, self.in_f, M))
            if self.b is not None and not bias_grad_done:
                K.colsum(dy_colsum if dy_colsum is not None else dy2d, self.b.grad)
        def dgrad():
            # dX = dY . W as an NT product on the transposed shadow W^T (in, out)
            if not need_dx:
                return None
            return K.gemm(dy2d, self.w.bf16_t, trans_b=True, out=dx_out, **dx_epi)
        if wgrad_overlap.active is None:
            wgrad()
            return dgrad()
        side, keep = wgrad_overlap.active
        keep.extend((dy2d, x2d, dy_colsum))
        # fork point before dX, dX issued first: the graph's first child of the fork is the
        # critical-path product, which keeps it on the main stream's hardware queue (issued after
        # the fork, it was queued behind the dW GEMM and its split-K combine on one queue)
        fork = torch.cuda.Event()
        fork.record(torch.cuda.current_stream())
        dx = dgrad()
        side.wait_event(fork)
        with torch.cuda.stream(side):
            wgrad()
        return dx


class SeqLayerNorm:
    """flax.linen.LayerNorm(reduction_axes=[1], feature_axes=[-1]) (vanilla_decoder.yaml:5-13)."""

    def __init__(self, store: ParamStore, name: str, D: int, eps: float = 1e-6):
        self.eps = eps
        self.scale = store.add(f"{name}/scale", (D,), const(1.0))
        self.bias = store.add(f"{name}/bias", (D,), const(0.0))

    def fwd(self, x):
        return K.seqnorm_fwd(x, self.scale.data, self.bias.data, self.eps)

    def bwd(self, dy, x, mean, rstd, addend=None, out=None):
        return K.seqnorm_bwd(dy, x, mean, rstd, self.scale.data, self.scale.grad, self.bias.grad,
                             addend=addend, out=out)
