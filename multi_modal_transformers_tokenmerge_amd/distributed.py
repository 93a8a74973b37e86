"""Data-parallel training over the GPUs of one node (one process per GPU, torch.distributed with
the "nccl" backend = RCCL over xGMI on ROCm).

The reference has no distributed code at all. Design here:
  * samples are independent (sequence LayerNorm, GroupNorm and ToMe are per sample), so the
    global batch is sharded: rank r owns global samples [r*B, (r+1)*B), and every random stream
    is keyed by the GLOBAL sample index (``sample_offset``), so N ranks x B reproduce 1 rank x N*B;
  * the only exchange is the gradient all-reduce over the flat fp32 gradient buffer, issued as a
    few large contiguous buckets (xGMI rings are per-link bound: few, large collectives); the
    1/N average is folded into the AdamW kernel's grad_scale instead of a separate pass;
  * the attention-dropout mask is keyed by (seed, step, layer) only, identical on every rank
    (Flax broadcasts it over the batch).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0

    @property
    def enabled(self) -> bool:
        return self.world_size > 1


def init_from_env(backend: str | None = None) -> DistInfo:
    """Initialise the process group from torchrun's environment (RANK/WORLD_SIZE/LOCAL_RANK/
    MASTER_ADDR/MASTER_PORT). Single process when WORLD_SIZE is unset or 1."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return DistInfo()
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:  # MMT_DIST_BACKEND=gloo: CPU-transport rehearsal of the multi-rank path
        backend = os.environ.get("MMT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return DistInfo(rank, ws, local)


class GradAllReducer:
    """All-reduce (SUM) of the flat gradient buffer in ``bucket_bytes`` contiguous slices.
    The average is applied by AdamW's grad_scale = 1 / world_size."""

    def __init__(self, world_size: int, bucket_bytes: int = 64 << 20, group=None):
        self.world_size = world_size
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.group = group

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world_size

    def __call__(self, flat_grad: torch.Tensor):
        if self.world_size <= 1:
            return
        n = flat_grad.numel()
        for s in range(0, n, self.bucket_elems):
            dist.all_reduce(flat_grad[s:s + self.bucket_elems], op=dist.ReduceOp.SUM, group=self.group)


class DDPStep:
    """One data-parallel training step of an Octo model on this rank's shard, as bench.py runs it:
    zero grads -> forward -> backward -> gradient all-reduce -> fused AdamW -> step counter.

    * world size 1: the whole step is ONE HIP graph (no host work between kernels);
    * world size N > 1: the backward runs as S block-range stages (Octo.backward_stage /
      stage_bounds; the heads and last blocks first; by default "auto": ~24 MB gradient regions
      from the top and a last stage of block 0 alone). After stage k the flat-gradient region it
      finalised (Octo.grad_regions) is all-reduced asynchronously on the collective stream while
      the later stages compute; AdamW (its own graph) waits for all of them, so only the last
      region (block 0 + the tokenizers / stem, exposed_bytes) is all-reduced with nothing to
      hide behind;
    * S = 1: one forward/backward graph, then a blocking bucketed all-reduce (GradAllReducer);
    * use_graph False: the same schedules launched eagerly (the overlap still applies).
    The 1/N average is AdamW's grad_scale (reducer.grad_scale)."""

    # Cross-step T5 pipeline (txt_next given): the frozen T5 encoder's output for the NEXT
    # step's text is computed on a side stream beside this step (the encoder has no trainable
    # parameter, so its output does not depend on this step's update), and the forward takes the
    # output computed one step earlier. Every step still runs exactly one T5 forward; it moves
    # from the head of the forward, where nothing else can run (the sequence assembly needs the
    # text), to beside the step's kernels. txt_next: the device buffer holding the NEXT step's
    # token ids when a step is called (a loader prefetching one batch ahead writes them there;
    # bench.py's synthetic batch repeats, so it passes txt itself). The first call after build()
    # (or after reset_text()) encodes the step's own `txt` before it starts, so a loader may
    # write the first batch after build(); from then on `txt` is not read for the encoder — each
    # step's text arrives through txt_next one call earlier (write both buffers, one batch apart).

    def __init__(self, model, state, txt, img, act, reducer: GradAllReducer | None = None,
                 stages="auto", use_graph: bool = True, txt_next=None):
        self.model, self.state = model, state
        self.txt, self.img, self.act = txt, img, act
        self.t5_pf = (txt_next is not None and txt is not None
                      and getattr(model, "t5", None) is not None)
        self.txt_next = txt_next
        self.t5_cur = self.t5_nxt = None
        self._t5_primed = False  # t5_cur holds T5(txt) of the coming step
        self._t5_side = torch.cuda.Stream(device=model.device) if self.t5_pf else None
        self._g_t5 = None
        self.reducer = reducer
        self.distributed = reducer is not None and reducer.world_size > 1
        # the backward's stage split (Octo.stage_bounds: an int, a list or "auto[:MB]")
        self.bounds = model.stage_bounds(stages) if self.distributed else [model.cfg.num_blocks, 0]
        self.S = len(self.bounds) - 1
        self.regions = model.grad_regions(self.bounds) if self.S > 1 else None
        self.use_graph = use_graph
        if self.distributed and getattr(state.allreduce, "grad_scale", 1.0) != reducer.grad_scale:
            # the 1/N average lives in AdamW's grad_scale (state.allreduce): a reducer given only
            # here would leave the gradients summed over the ranks, never averaged
            raise ValueError("DDPStep: pass the same GradAllReducer to create_octo_train_state "
                             "(state.allreduce) so AdamW averages the summed gradients")
        self.loss_buf = torch.zeros(1, device=model.device)
        self.graphs = []
        self._st = {}

    # --------------------------------------------------------------- schedule pieces
    def _t5_prime(self):
        """The first step's T5 output (outside the timed steps: the one encoder run the pipeline
        moves ahead of step 1)."""
        if self.t5_pf and self.t5_cur is None:
            self.t5_cur = self.model.t5(self.txt).clone()
            self.t5_nxt = torch.empty_like(self.t5_cur)

    def reset_text(self):
        """The next call encodes its own `txt` again instead of the encoder output handed over by
        the previous call (e.g. after the loader restarted, or `txt` was rewritten alone)."""
        self._t5_primed = False

    def _t5_first_call(self):
        if self.t5_pf and not self._t5_primed:
            self.t5_cur.copy_(self.model.t5(self.txt))
            self._t5_primed = True

    def _t5_fork(self):
        """Next step's T5 on the side stream, all of it launched here."""
        side = self._t5_side
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self.t5_nxt.copy_(self.model.t5(self.txt_next))

    def _t5_join(self):
        """After the backward (the text projection's dW read t5_cur): the next output becomes
        the current one."""
        torch.cuda.current_stream().wait_stream(self._t5_side)
        self.t5_cur.copy_(self.t5_nxt)

    # where the next step's encoder runs (benchmarking knob MMT_T5_FORK): "ext" (default) its own
    # graph replayed on the side stream right before the step's graph(s), handed over after the
    # backward; "fwd" / "bwd" forked inside the step's graph at its start / after the forward.
    # "ext" and "fwd" measure the same, "bwd" and forks between the forward's blocks less
    # (profiles/r05_t5_overlap_ab.txt); "ext" leaves the step's graphs as they are without it.
    t5_fork_at = os.environ.get("MMT_T5_FORK", "ext")

    @property
    def _t5_graphed_in(self):
        return self.t5_pf and self.t5_fork_at in ("fwd", "bwd")

    def _fwd_bwd(self):
        m, s = self.model, self.state
        m.store.zero_grad()
        early = self._t5_graphed_in and self.t5_fork_at == "fwd"
        if early:
            self._t5_fork()
        loss, st = m.compute_diffusion_denoise_loss(self.txt, self.img, self.act, True, s.rng,
                                                    s.sample_offset, t5_out=self.t5_cur)
        if self._t5_graphed_in and not early:
            self._t5_fork()
        m.backward(st)
        if self._t5_graphed_in:
            self._t5_join()
        self.loss_buf.copy_(loss)

    def _t5_ext_launch(self):
        """"ext": the next step's encoder on the side stream, after everything before this step
        (the previous hand-over included) and beside the step's graph."""
        if self.t5_pf and not self._t5_graphed_in:
            side = self._t5_side
            side.wait_stream(torch.cuda.current_stream())
            if self._g_t5 is not None:
                with torch.cuda.stream(side):
                    self._g_t5.replay()
            else:
                self._t5_fork()

    def _t5_ext_join(self):
        if self.t5_pf and not self._t5_graphed_in:
            self._t5_join()

    def _stage(self, k):
        m, s = self.model, self.state
        early = self._t5_graphed_in and self.t5_fork_at == "fwd"
        if k == 0:
            m.store.zero_grad()
            if early:
                self._t5_fork()
            loss, st = m.compute_diffusion_denoise_loss(self.txt, self.img, self.act, True, s.rng,
                                                        s.sample_offset, t5_out=self.t5_cur)
            self.loss_buf.copy_(loss)
            self._st["st"] = st
            if self._t5_graphed_in and not early:
                self._t5_fork()
        m.backward_stage(self._st["st"], k, self.bounds)
        if self._t5_graphed_in and k == 0:  # joined inside the stage's graph (self-contained)
            torch.cuda.current_stream().wait_stream(self._t5_side)
        if self._t5_graphed_in and k == self.S - 1:  # after the text projection's dW
            self.t5_cur.copy_(self.t5_nxt)

    def _opt(self):
        self.state.apply_gradients()

    @property
    def exposed_bytes(self) -> int:
        """fp32 gradient bytes all-reduced after the backward's last stage (not overlapped)."""
        if not self.distributed:
            return 0
        lo, hi = self.regions[-1] if self.regions else (0, self.model.store.n)
        return 4 * (hi - lo)

    def _reduce_async(self, k):
        lo, hi = self.regions[k]
        return dist.all_reduce(self.model.store.flat_grad[lo:hi], op=dist.ReduceOp.SUM,
                               async_op=True, group=self.reducer.group)

    # --------------------------------------------------------------------- capture
    def _snapshot(self):
        st, s = self.model.store, self.state
        snap = [t.clone() for t in (st.flat, st.flat_bf16, st.m, st.v, s.rng)]
        if s.metrics is not None:
            snap += [s.metrics.total.clone(), s.metrics.count.clone()]
        return snap

    def _restore(self, snap):
        st, s = self.model.store, self.state
        dst = [st.flat, st.flat_bf16, st.m, st.v, s.rng]
        if s.metrics is not None:
            dst += [s.metrics.total, s.metrics.count]
        for d, v in zip(dst, snap):
            d.copy_(v)
        st.refresh_transposed()
        st.refresh_fp8()

    def build(self, warm: int = 2):
        """Warm caches and the allocator outside capture, then capture the step's graphs. The
        warm-up steps train: parameters, AdamW moments, the step counter and the metrics are
        snapshotted before them and restored after, so build() leaves the training state as it
        found it (the captured graphs then start from that state; the transposed and e4m3 weight
        shadows are re-derived from the restored bf16 shadow; tests/test_train_state_gpu.py
        checks every buffer bitwise). The snapshot holds one extra copy of the fp32 master, the
        bf16 shadow and both AdamW moments during build(): 14 bytes per parameter (≈ 315 MB for
        OCTO-small's 22.5 M, ≈ 1.2 GB for OCTO-base), freed before capture."""
        self._t5_prime()
        if not self.use_graph:
            return self
        snap = self._snapshot()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warm):
                self._fwd_bwd()
                if self.distributed:
                    self.reducer(self.model.store.flat_grad)
                self._opt()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self._restore(snap)
        del snap
        self._t5_primed = False  # the first call encodes the txt it finds then
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()

        def cap(fn):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                fn()
            self.graphs.append(g)
        if self.t5_pf and not self._t5_graphed_in:  # "ext": the encoder's own graph (own pool:
            side = self._t5_side                       # it replays beside the step's graphs)
            side.wait_stream(torch.cuda.current_stream())
            self._g_t5 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._g_t5, stream=side):
                self.t5_nxt.copy_(self.model.t5(self.txt_next))
            torch.cuda.current_stream().wait_stream(side)
        if self.S > 1:
            for k in range(self.S):   # one graph per backward stage (the first holds the forward)
                cap(lambda k=k: self._stage(k))
            cap(self._opt)
        elif self.distributed:
            cap(self._fwd_bwd)
            cap(self._opt)
        else:
            def whole():
                self._fwd_bwd()
                self._opt()
            cap(whole)
        return self

    def __call__(self):
        g = self.graphs
        self._t5_prime()
        self._t5_first_call()
        self._t5_ext_launch()
        if self.S > 1:
            works = []
            for k in range(self.S):
                g[k].replay() if self.use_graph else self._stage(k)
                works.append(self._reduce_async(k))
            self._t5_ext_join()
            for w in works:
                w.wait()
            g[self.S].replay() if self.use_graph else self._opt()
        elif self.distributed:
            g[0].replay() if self.use_graph else self._fwd_bwd()
            self._t5_ext_join()
            self.reducer(self.model.store.flat_grad)
            g[1].replay() if self.use_graph else self._opt()
        else:
            if self.use_graph:
                g[0].replay()
            else:
                self._fwd_bwd()
                self._opt()
            self._t5_ext_join()
