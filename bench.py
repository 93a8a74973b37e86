#!/usr/bin/env python3
"""Benchmark of the hot path: train samples/sec of the OCTO-small diffusion training step
(256x256 image + 32-token text, ToMe r=16 per block, bf16 MFMA) on N MI355X — BASELINE.json's
metric, config[2] (the single-GPU line uses the same workload at N=1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config NAME]
    torchrun --nproc-per-node N bench.py --gpus N ...          (one process per GPU, RCCL)

Per-GPU batch 512 by default (round-2 sweep on one MI355X: 11.4k / 12.3k / 12.7k / 12.8k / 13.4k /
13.6k / 13.8k samples/s at B = 192 / 256 / 320 / 384 / 512 / 768 / 1024; fixed per-step costs —
cross-queue waits, small launches, AdamW — amortise; see DESIGN.md "Batch").
One step = zero grads -> forward (frozen T5, image stem, 12 ToMe blocks, diffusion loss) ->
backward -> [gradient all-reduce over RCCL] -> fused AdamW -> device step counter, on synthetic
inputs resident in HBM (numpy default_rng(0) shapes of SURVEY §8d). The N=1 step is one HIP graph
replay; with N>1 the backward runs as --overlap-stages graphs (default auto: ~24 MB gradient
regions, block 0 alone last), each stage's gradient
region all-reduced asynchronously on the RCCL stream while the later stages compute, and the AdamW
graph waits for them (distributed.DDPStep; --no-graph launches the same schedule eagerly).
Timing: barrier + synchronize on both sides of exactly K steps, max over ranks.

Printed on rank 0: ONE JSON line with the metric, a roofline object for the dominant kernel
(MFMA GEMM of the MLP up-projection, measured here with HIP events on its own stream) and the
CPU baseline (the fp32 CPU restatement oracle/octo_ref.py, a bounded sample on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multi_modal_transformers_tokenmerge_amd import _kernels as K  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.distributed import (  # noqa: E402
    DDPStep, GradAllReducer, init_from_env)
from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.models.octo.octo import (  # noqa: E402
    Octo, create_octo_train_state)

MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md, chip table)
MFMA_FP8_PEAK_TFLOPS = 5000.0    # MI355X dense fp8 (e4m3; the 10 PF figure is 2:1 sparsity)
HBM_PEAK_GBS = 8000.0


def synthetic_inputs(model, B, rank, device):
    cfg = model.cfg
    g = np.random.default_rng(rank)
    H = cfg.image_size[0]
    img = torch.from_numpy(g.integers(0, 256, (B, model.n_images, H, H, 3), dtype=np.uint8)).to(device)
    txt = (torch.from_numpy(g.integers(0, cfg.t5.vocab_size, (B, model.n_text), dtype=np.int32)).to(device)
           if model.has_text else None)
    act = torch.from_numpy(g.uniform(-1, 1, (B, cfg.action_space_dim)).astype(np.float32)).to(device)
    return txt, img, act


def algorithmic_flops_per_sample(model) -> float:
    """SURVEY §8d formula: trainable ops 3x forward (fwd + 2x bwd), frozen T5 1x."""
    cfg = model.cfg
    D, M = cfg.token_embedding_dim, cfg.mlp_dim
    tr = 0.0
    for (sets, _, ts, r, prune, _plan) in model.layer_sets:
        L = sets.L
        if prune is None:   # ToMe merges after the out-projection
            Lp = L - r
            tr += 2 * L * 4 * D * D + 2 * Lp * 2 * D * M + 4 * L * L * D
        else:               # pruning happens before it
            Lp = sum(prune[1])
            tr += 2 * L * 3 * D * D + 2 * Lp * D * D + 2 * Lp * 2 * D * M + 4 * L * L * D
    stem = 0.0
    rs = model.image_tokenizer.resnet
    npat = model.image_tokenizer.num_patches * model.n_images
    stem += 2 * npat * rs.win * (rs.kh * rs.kw * 3) * 64 + npat * (2 * 2 * 64 * 64 + 2 * 64 * D)
    t5 = 0.0
    if model.has_text:
        c = cfg.t5
        T = model.n_text
        per_tok = 2 * (4 * c.d_model * c.num_heads * c.d_kv + 2 * c.d_model * c.d_ff)
        t5 = c.num_layers * (T * per_tok + 4 * T * T * c.num_heads * c.d_kv)
        if model.text_proj is not None:
            tr += 2 * T * c.d_model * D
    return 3 * (tr + stem) + t5


PROBE_KERNEL = "gemm_xs_kernel<false, true>"  # the MLP up (relu-bit image) at K = 384
NT256_KERNEL = "gemm_nt256_kernel<256, 0, 0, 2, false, false, false>"


def _graph_time_us(launch, reps):
    """Average duration of `launch` (µs): reps launches captured in one HIP graph (no host gaps,
    as in the training step), timed with HIP events recorded on the stream the graph replays on."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            launch()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            launch()
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def _gemm_bytes(M, N, K, out_bytes=2, extra=0):
    return 2 * (M * K + N * K) + out_bytes * M * N + extra


def kernel_probes(model, B, reps=20):
    """The step's heaviest kernels at their exact block-0 shapes (B per GPU), each launched alone:
    per probe the kernel name (rocprofv3 substring), the average launch duration and the
    algorithmic work per launch (flops for MFMA-bound kernels, bytes for HBM-bound ones; DESIGN.md
    §3 states each figure). Covers the top of the step's trace: the nt256 GEMM (MLP up), the
    direct-to-LDS NT GEMM (MLP input gradient, N = 384, K = 1536), the split-K weight-gradient
    GEMM (MLP Dense_0 dW), attention forward and backward (dQ + dK/dV), ToMe matching, the merge
    forward alone and fused with LayerNorm_1 (the form the step runs), the fused LN_1 backward +
    unmerge + dropout backward, and the sequence-axis LayerNorm forward and backward."""
    from multi_modal_transformers_tokenmerge_amd.layers import split_k_for
    cfg = model.cfg
    dev = model.device
    blk = model.stack.blocks[0]
    sets, table, ts, r, prune, plan = model.layer_sets[0]
    L = sets.L
    L1 = sum(prune[1]) if prune else L - r
    D, Mh, H = cfg.token_embedding_dim, cfg.mlp_dim, cfg.num_heads
    Dh = D // H
    g = torch.Generator(device="cpu").manual_seed(0)

    def rnd(*shape, dt=torch.bfloat16):
        return torch.randn(shape, generator=g).to(dt).to(dev)

    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    out = []

    def add(name, kernel, launch, bound, work, note, alg_bytes=None):
        us = _graph_time_us(launch, reps)
        if bound in ("mfma", "mfma8"):
            ach = work / (us * 1e-6) / 1e12
            peak = MFMA_FP8_PEAK_TFLOPS if bound == "mfma8" else MFMA_BF16_PEAK_TFLOPS
            out.append(dict(name=name, kernel=kernel, bound="mfma", avg_launch_us=round(us, 2),
                            flops_per_launch=work, achieved=round(ach, 2),
                            peak=peak, unit="TFLOP/s", dtype="fp8" if bound == "mfma8" else "bf16",
                            frac=round(ach / peak, 4), note=note,
                            algorithmic_bytes_per_launch=alg_bytes))
        else:
            ach = work / (us * 1e-6) / 1e9
            out.append(dict(name=name, kernel=kernel, bound="hbm", avg_launch_us=round(us, 2),
                            bytes_per_launch=work, achieved=round(ach, 1), peak=HBM_PEAK_GBS,
                            unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4), note=note))

    # 1. MLP up-projection (bias + relu + dropout epilogue + the relu-bit image the backward
    # gates with, as the step launches it)
    M = B * L1
    y1 = rnd(M, D)
    h = torch.empty((M, Mh), dtype=torch.bfloat16, device=dev)
    hb = (torch.empty((-(-M // 256) * 256, Mh // 32), dtype=torch.int32, device=dev)
          if K.gemm_bits_supported(M, Mh, D) and not blk.mlp.dense.fp8 else None)
    up_kernel = ("gemm_xs_kernel<true" if blk.mlp.dense.fp8 else
                 PROBE_KERNEL if D == 384 else NT256_KERNEL)  # fp8: e4m3 on the XS kernel (+ quant)
    add("mlp_up_fwd", up_kernel,
        lambda: blk.mlp.dense.fwd(y1, out=h, act=K.ACT_RELU, rng=rng, drop_layer=0, drop_site=2,
                                  keep_prob=0.9, relu_bits=hb),
        "mfma", 2.0 * M * Mh * D, f"M={M} N={Mh} K={D}, 2MNK (+ bias, relu, dropout, relu bits)",
        _gemm_bytes(M, Mh, D, extra=4 * Mh) + (M * Mh // 8 if hb is not None else 0))
    # 1b. fp8 weight path (BASELINE configs[4]): the same product in e4m3 on
    # v_mfma_scale_f32_32x32x64_f8f6f4 (per-row activation / per-channel weight scales), priced
    # against the dense fp8 peak; its bf16 twin is mlp_up_fwd above (same shape and epilogue)
    if blk.mlp.dense.fp8:
        yq, sy = K.quant_rows_fp8(y1)
        w8 = blk.mlp.dense.w
        b8 = blk.mlp.dense.b.data
        add("mlp_up_fwd_fp8", "gemm_xs_kernel<true",
            lambda: K.gemm_fp8(yq, sy, w8.q8, w8.q8_scale, out=h, bias=b8, act=K.ACT_RELU, rng=rng,
                               drop_layer=0, drop_site=2, keep_prob=0.9),
            "mfma8", 2.0 * M * Mh * D, f"M={M} N={Mh} K={D}, 2MNK in e4m3 (+ bias, relu, dropout; "
            "the activation quantisation is its own kernel)", M * D + Mh * D + 2 * M * Mh + 4 * (M + Mh))
        add("mlp_up_fwd_bf16_twin", PROBE_KERNEL if D == 384 else NT256_KERNEL,
            lambda: K.gemm(y1, w8.bf16, trans_b=True, out=h, bias=b8, act=K.ACT_RELU, rng=rng,
                           drop_layer=0, drop_site=2, keep_prob=0.9),
            "mfma", 2.0 * M * Mh * D, f"M={M} N={Mh} K={D}: the fp8 probe's product in bf16 (A/B)",
            _gemm_bytes(M, Mh, D, extra=4 * Mh))
    # 2. MLP input gradient dy1 = dz1 . W1 (NT on the transposed shadow): N = 384, K = 1536 — a
    # plain narrow product: gemm_ntw_kernel
    dz1 = rnd(M, Mh)
    dy1 = torch.empty((M, D), dtype=torch.bfloat16, device=dev)
    add("mlp_dx", "gemm_ntw_kernel",
        lambda: K.gemm(dz1, blk.mlp.dense.w.bf16_t, trans_b=True, out=dy1),
        "mfma", 2.0 * M * D * Mh,
        f"M={M} N={D} K={Mh}, 2MNK (one or two launches of the narrow-output NT kernel)",
        _gemm_bytes(M, D, Mh))
    # 3. MLP Dense_0 weight gradient dW += dz1^T . y1 (TN, split-K fp32 slabs + combine); the
    # standalone probe splits for the whole chip (256 workgroups), the step's launches for half of
    # it (layers.split_k_for: they share the CUs with the main queue)
    wgrad = torch.zeros((Mh, D), dtype=torch.float32, device=dev)
    sk = split_k_for(Mh, D, M, wgs=256)
    add("mlp_dw", "gemm_tn_dma16_kernel",
        lambda: K.gemm(dz1, y1, trans_a=True, out=wgrad, out_mode=K.OUT_F32_ACCUM, split_k=sk),
        "mfma", 2.0 * M * D * Mh,
        f"M={Mh} N={D} K={M}, 2MNK, split-K {sk} (the GEMM + its combine kernel together; "
        "full-chip split, the step splits for 128 workgroups)",
        2 * (M * Mh + M * D) + 8 * Mh * D)
    # 3b./3c. the residual-stream products (fp32 out = fp32 residual + dropout(x W^T + b)):
    # MLP Dense_1 and the attention out-projection of block 0 (reference attention.py:36-37,
    # 59-63). HBM-bound: algorithmic bytes = A (bf16) + W (bf16) read, residual (fp32) read,
    # out (fp32) written; the bias is negligible
    for name, rows, kin, dn in (("res_dense1", M, Mh, blk.mlp.dense_out),
                                ("res_outproj", B * L, D, blk.out)):
        a_in = rnd(rows, kin)
        res_in = rnd(rows, D, dt=torch.float32)
        out_f = torch.empty((rows, D), dtype=torch.float32, device=dev)
        add(name, "gemm_glds_nt_kernel",
            lambda a_in=a_in, res_in=res_in, out_f=out_f, dn=dn: dn.fwd(
                a_in, out=out_f, out_mode=K.OUT_F32, residual=res_in, rng=rng, drop_layer=0,
                drop_site=3, keep_prob=0.9),
            "hbm", 2 * (rows * kin + D * kin) + 8 * rows * D,
            f"M={rows} N={D} K={kin}: read A bf16 + W bf16 + residual fp32, write C fp32")
    # 4./5. attention forward and backward of block 0 (token-set mask, dropout)
    qkv = rnd(B, L, 3 * D)
    kpa = 1.0 - cfg.attention_dropout_rate
    bits = K.dropout_bits(rng, 0, 0, L, L, kpa)
    scale = Dh ** -0.5
    o, lse = K.attn_fwd(qkv, H, scale, table, bits, kpa)
    fwd_flops = 4.0 * L * L * Dh * H * B
    add("attn_fwd", "attn_fwd_res_kernel" if K.attn_fwd_resident(L, Dh) else "attn_fwd_kernel",
        lambda: K.attn_fwd(qkv, H, scale, table, bits, kpa), "mfma", fwd_flops,
        f"B={B} L={L} H={H} Dh={Dh}: 4 L^2 Dh H B (dense count, masked tiles included)",
        B * L * (3 * D + D) * 2 + B * H * L * 4)
    do = rnd(B, L, D)
    bgrad = torch.zeros(3 * D, dtype=torch.float32, device=dev)
    res_b = K.attn_bwd_resident(L, Dh)
    add("attn_bwd", "attn_bwd_res" if res_b else "attn_bwd_dkdv_kernel",  # res / res8 kernels
        lambda: K.attn_bwd(qkv, o, do, lse, H, scale, table, bits, kpa, bias_grad=bgrad),
        "mfma", 2.5 * fwd_flops,
        ("one resident kernel (dQ beside dK / dV)" if res_b else "dQ + dK/dV kernels together")
        + ": 2.5 x the forward count (flash-attention convention)",
        B * L * (3 * D + 2 * D + 3 * D) * 2 + B * H * L * 8)
    # 6. ToMe matching and merge forward of block 0 (metric = K of the image set, fp32 residual)
    if r > 0:
        # the first (set, r) of block 0's merge plan: with several merged sets (ts == -2) r is
        # their sum, so probe one set with its own r (the step runs one match + merge per set)
        si, r = plan[0]
        s0, t = sets.starts[si], sets.lens[si]
        x1 = rnd(B, L, D, dt=torch.float32)
        metric = qkv.view(B, L, 3, H, Dh)[:, s0:s0 + t, 1]
        add("tome_match", "tome_match_fused_kernel",
            lambda: K.tome_match(metric, r), "hbm",
            B * t * H * Dh * 2 + B * ((t + 1) // 2) * 4,
            "read the K rows of the set (all heads), write src/dst/unm indices")
        unm, src, dst = K.tome_match(metric, r)
        torch.cuda.synchronize()
        add("tome_merge_fwd", "tome_merge_fwd_kernel",
            lambda: K.tome_merge_fwd(x1, s0, t, r, unm, src, dst, size_in=None), "hbm",
            B * L * D * 4 + B * (L - r) * D * 4 + B * (t - r) * 4,
            "read the fp32 sequence, write the merged sequence and the token sizes")
        # 6b. what the step actually runs after the attention residual: the ToMe merge fused with
        # LayerNorm_1's forward (one pass: merged fp32 sequence, sizes, pos_map, y bf16, stats)
        gam = torch.ones(D, device=dev)
        bet = torch.zeros(D, device=dev)
        nidx = (t + 1) // 2 + r           # unm + src + dst indices read
        if L - r <= 512:  # the fused forms' shapes (attention_blocks/attention.py uses them there)
            add("tome_merge_seqnorm_fwd", "tome_merge_seqnorm_fwd_kernel",
                lambda: K.tome_merge_seqnorm_fwd(x1, s0, t, r, unm, src, dst, gam, bet, 1e-6),
                "hbm", B * L * D * 4 + B * (L - r) * D * (4 + 2) + B * (t - r) * 4 + B * t * 4
                + 2 * B * D * 4 + B * nidx * 4,
                "read the fp32 sequence; write the merged sequence (fp32), LN_1 output (bf16), sizes, "
                "pos_map and the LN statistics (token_compression.py:90-129 + attention.py:66)")
            # 6c. its backward: LayerNorm_1 backward + unmerge + attention-output dropout backward
            xm, so, pos, _, mu1, rs1 = K.tome_merge_seqnorm_fwd(x1, s0, t, r, unm, src, dst, gam, bet, 1e-6)
            L2 = L - r
            dy1 = rnd(B, L2, D)
            dx2 = rnd(B, L2, D, dt=torch.float32)
            ggam, gbet, gb = (torch.zeros(D, device=dev) for _ in range(3))
            if K.ln_unmerge_ok(L, L2):
                add("ln_unmerge_dropout_bwd", "ln_unmerge_dropout_bwd_kernel",
                    lambda: K.ln_unmerge_dropout_bwd(dy1, xm, mu1, rs1, gam, ggam, gbet, dx2,
                                                     (s0, t, r, pos, None, so), rng, 0, 1, 0.9, 0,
                                                     bias_grad=gb),
                    "hbm", B * L2 * D * (2 + 4 + 4) + B * L * D * (4 + 2) + B * t * 4 + B * (t - r) * 4
                    + 2 * B * D * 4,
                    "read dy (bf16), x and the residual gradient (fp32); write the unmerged gradient "
                    "(fp32) and the dropout output (bf16)")
    # 7. sequence-axis LayerNorm forward (fp32 residual stream -> bf16) and backward
    x = rnd(B, L1, D, dt=torch.float32)
    add("seqnorm_fwd", "seqnorm_fwd_kernel", lambda: blk.ln1.fwd(x), "hbm",
        B * L1 * D * (4 + 2) + 2 * B * D * 4, "read x (fp32); write y (bf16) and mean / rstd")
    _, mu, rs = blk.ln1.fwd(x)
    dy = rnd(B, L1, D)
    addend = rnd(B, L1, D, dt=torch.float32)
    add("seqnorm_bwd", "seqnorm_bwd_kernel",
        lambda: blk.ln1.bwd(dy, x, mu, rs, addend=addend), "hbm", B * L1 * D * (4 + 2 + 4 + 4),
        "read x (fp32), dy (bf16), the addend (fp32); write dx (fp32)")
    return out


def source_digest() -> str:
    """sha256 of the kernel sources (csrc/*.hip, csrc/*.h, include/*.h): identifies the code a
    PMC traffic pass measured, independent of rebuilds of the same sources."""
    import glob
    import hashlib
    h = hashlib.sha256()
    pkg = os.path.join(ROOT, "multi_modal_transformers_tokenmerge_amd", "csrc")
    files = sorted(glob.glob(os.path.join(pkg, "*.hip")) + glob.glob(os.path.join(pkg, "*.h"))
                   + glob.glob(os.path.join(ROOT, "include", "*.h")))
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def probe_traffic(B: int):
    """HBM bytes per launch of each probe from the committed rocprofv3 PMC passes
    (profiles/*_probe_pmc.json, written by tools/pmc_traffic.py from a FETCH_SIZE and a WRITE_SIZE
    pass over `bench.py --probe-only`: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md "HBM"): only a file measured at this per-GPU batch on kernel sources with
    this source_digest() counts (a pass over other code is stale: its probes report traffic
    null). Returns ({name: bytes}, file name or None)."""
    import glob
    found, src, dig = {}, None, source_digest()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_probe_pmc.json"))):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("batch", 256) == B and d.get("source_digest") == dig:
            found = {k: v["hbm_bytes_per_launch"] for k, v in d.get("probes", {}).items()}
            src = os.path.basename(f)
    return found, src


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def _cpu_run(cfg_name, model, train=True, budget_s=20.0, B=8, max_steps=10):
    """The fp32 CPU restatement (oracle/octo_ref.py) on `model`'s parameters: one warm-up step,
    then up to `max_steps` steps within `budget_s`; (samples/s from the MEDIAN step time, steps,
    median s). train: forward + backward + AdamW; else the forward (loss) alone."""
    from oracle.octo_ref import OctoRef, sequence_spec
    cfg = model.cfg
    params = {p.name: p.data.detach().float().cpu().clone().requires_grad_(train)
              for p in model.store.params}
    t5p = ({p.name: p.bf16.float().cpu() for p in model.t5.store.params} if model.has_text else None)
    ref = OctoRef(cfg, params, t5p)
    opt = torch.optim.AdamW(list(params.values()), lr=3e-4, weight_decay=1e-4) if train else None
    g = np.random.default_rng(0)
    H = cfg.image_size[0]
    images = g.integers(0, 256, (B, model.n_images, H, H, 3)).astype(np.float32)
    text = g.integers(0, cfg.t5.vocab_size, (B, model.n_text)).astype(np.int32) if model.has_text else None
    actions = g.uniform(-1, 1, (B, cfg.action_space_dim)).astype(np.float32)
    npat = model.image_tokenizer.num_patches * model.n_images
    pos = (g.integers(0, 127, (B, npat)), g.integers(0, 127, (B, npat)))
    spec = sequence_spec(cfg.input_sequence, cfg.token_compression_sequence)

    def step(i):
        with torch.set_grad_enabled(train):
            if train:
                opt.zero_grad(set_to_none=True)
            loss, _ = ref.forward_loss(text, images, actions, seed=1, step=i, positions=pos,
                                       t=g.integers(0, cfg.diffusion_steps, B),
                                       eps=g.standard_normal((B, cfg.action_space_dim)).astype(np.float32),
                                       sequence=spec)
            if train:
                loss.backward()
                opt.step()
    step(0)  # warm-up
    times, t_all = [], time.perf_counter()
    while len(times) < max_steps and time.perf_counter() - t_all < budget_s:
        t0 = time.perf_counter()
        step(len(times) + 1)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return B / med, len(times), med


def cpu_baseline(cfg_name, model, budget_s=20.0, B=8, max_steps=10):
    """fp32 CPU restatement (oracle/octo_ref.py) forward+backward+AdamW on a bounded sample of the
    same workload: B = 8, median step time (_cpu_run). Threads: torch's intra-op
    pool (the box sets OMP_NUM_THREADS to its CPU share), reported as `cores`. `other` carries
    SURVEY §8d's other two CPU samples — OCTO-tiny forward only and OCTO-small r = 0 training —
    on smaller budgets (≈ 5 s each; CPU-built models, same restatement)."""
    threads = torch.get_num_threads()
    v, n, med = _cpu_run(cfg_name, model, True, budget_s, B, max_steps)
    other = []
    for name, train, b, budget, steps in (("octo-tiny", False, 8, 3.0, 5), ("octo-small", True, 8, 5.0, 3)):
        try:
            m = Octo(get_config(name), torch.device("cpu"), seed=0)
            ov, on, omed = _cpu_run(name, m, train, budget, b, steps)
            other.append(dict(config=name, mode="fwd+bwd+AdamW" if train else "forward", batch=b,
                              value=round(ov, 3), unit="samples/s", steps=on,
                              median_s_per_step=round(omed, 3)))
        except Exception as e:  # a baseline sample must never sink the bench line
            other.append(dict(config=name, error=f"{type(e).__name__}: {e}"))
    return dict(value=v, unit="samples/s", cores=threads, kind="port",
                sample=f"{cfg_name} fp32 torch-CPU restatement (oracle/octo_ref.py), fwd+bwd+AdamW "
                       f"at B={B}: median of {n} steps after 1 warm-up ({med:.2f} s/step) on "
                       f"{threads} threads of {_cpu_model()} (the JAX reference is not importable "
                       "offline)", other=other)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)   # 100 timed, 20 warm-up
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512,
                    help="per-GPU batch (512: see DESIGN.md 'Batch'; 64 leaves the chip underfilled)")
    ap.add_argument("--config", default="octo-small-tome16")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="config override (A/B runs), e.g. --set fp8=0 on octo-base-hires-tome32")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--overlap-stages", default="auto",
                    help="N > 1: backward stages, each stage's gradient region all-reduced while "
                         "the rest of the backward runs: an int (block ranges; 1 = no overlap) or "
                         "auto[:MB] (~MB-megabyte regions, default 24, block 0 alone last)")
    ap.add_argument("--deterministic", action="store_true",
                    help="bitwise-reproducible gradients (fixed-point shadow instead of fp32 "
                         "atomics; same as MMT_DETERMINISTIC=1)")
    ap.add_argument("--no-probes", action="store_true",
                    help="skip the per-kernel roofline probes (rocprofv3 traces of the step alone)")
    ap.add_argument("--probe-only", action="store_true",
                    help="only launch the dominant GEMM (for rocprofv3 --pmc traffic passes)")
    args = ap.parse_args()

    di = init_from_env()
    N = di.world_size
    if args.gpus != N and N > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {N}", file=sys.stderr)
    # (local_rank modulo the visible devices: lets a 2-rank gloo rehearsal share one GPU)
    dev = torch.device("cuda", di.local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    over = {}
    for kv in args.set:
        k, v = kv.split("=", 1)
        over[k] = (v.lower() in ("1", "true", "yes")) if v.lower() in ("0", "1", "true", "false", "yes", "no") \
            else (int(v) if v.lstrip("-").isdigit() else v)
    cfg = get_config(args.config, **over)
    B = args.batch
    if args.deterministic:
        os.environ["MMT_DETERMINISTIC"] = "1"
    model = Octo(cfg, dev, seed=0)
    if args.probe_only:  # for rocprofv3 --pmc traffic passes (tools/pmc_traffic.py)
        print(json.dumps(dict(probe_only=True, batch=B, source_digest=source_digest(),
                              probes=kernel_probes(model, B))), flush=True)
        return
    if di.enabled:  # identical initial parameters on every rank (broadcast from rank 0)
        dist.broadcast(model.store.flat, 0)
        model.store.sync_shadow()
    reducer = GradAllReducer(N) if di.enabled else None
    state = create_octo_train_state(model, seed=1234, allreduce=reducer, sample_offset=di.rank * B)
    txt, img, act = synthetic_inputs(model, B, di.rank, dev)
    use_graph = not args.no_graph
    # N > 1: the backward runs as --overlap-stages block-range stages, each stage's gradient
    # region all-reduced asynchronously while the later stages compute (distributed.DDPStep)
    ov = args.overlap_stages
    # the frozen T5 encoder of the next step's text runs beside this step's backward (one T5
    # forward per step either way; the synthetic batch repeats, so the next text is txt)
    t5_pipe = model.has_text and os.environ.get("MMT_T5_PIPELINE", "1") != "0"
    step = DDPStep(model, state, txt, img, act, reducer, stages=int(ov) if ov.isdigit() else ov,
                   use_graph=use_graph, txt_next=txt if t5_pipe else None).build()
    loss_buf = step.loss_buf

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if di.enabled:
        dist.barrier()
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(cur)
    host_s = 0.0  # host time inside step() (the graph launch enqueues every node from the CPU)
    for i in range(args.steps):
        h0 = time.perf_counter()
        step()
        host_s += time.perf_counter() - h0
        evs[i + 1].record(cur)  # step boundaries (a step ends with AdamW on this stream)
    torch.cuda.synchronize()
    if di.enabled:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if di.enabled:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss_val = float(loss_buf.item())
    K.device_status()  # after the timed region: no device-side index check fired in any step

    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]
    if di.rank == 0:
        ms = elapsed / args.steps * 1e3
        value = N * B * args.steps / elapsed
        probes = [] if args.no_probes else kernel_probes(model, B)
        traffic, traffic_src = probe_traffic(B)
        for pr in probes:
            pr["traffic"] = traffic.get(pr["name"])
        # headline: the dominant kernel of the step trace — the weight-gradient GEMM (TN, split-K
        # slabs + combine; ≈ 23 % of kernel time, profiles/r02_b512_kernel_stats_step.csv), at
        # the MLP Dense_0 dW shape; every other probe follows in `kernels`
        top = next((p for p in probes if p["name"] == "mlp_dw"), None)
        sets0, _, _, r0, pr0, _plan0 = model.layer_sets[0]
        M_ = B * (sum(pr0[1]) if pr0 else sets0.L - r0)
        N_, K_ = cfg.mlp_dim, cfg.token_embedding_dim
        if top is None:
            top = dict(achieved=None, frac=None, traffic=None, kernel="gemm_tn_dma16_kernel",
                       avg_launch_us=None, flops_per_launch=None)
        roof = dict(bound="mfma", achieved=top["achieved"], peak=MFMA_BF16_PEAK_TFLOPS,
                    unit="TFLOP/s", frac=top["frac"], traffic=top["traffic"],
                    kernel=top["kernel"] + " + splitk_epilogue_kernel<1> (MLP Dense_0 weight "
                    "gradient dW += dz1^T . y1: one mmt_gemm launch, split-K GEMM and its combine "
                    "timed together)",
                    shape_MNK=[N_, K_, M_], avg_launch_us=top["avg_launch_us"],
                    flops_per_launch=top["flops_per_launch"],
                    algorithmic_bytes_per_launch=2 * (M_ * N_ + M_ * K_) + 8 * N_ * K_,
                    traffic_source=(f"profiles/{traffic_src} (source digest {source_digest()})"
                                    if traffic_src else "no PMC pass of these kernel sources "
                                    f"(digest {source_digest()}): traffic null"),
                    kernels=[p for p in probes if p is not top])
        fps = algorithmic_flops_per_sample(model)
        cpu = None
        if N == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.config, model, budget_s=args.cpu_budget)
        sets0 = model.layer_sets[0][0]
        line = {
            "metric": "train samples/sec OCTO-small 256px+text, ToMe r=16, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "samples/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "median_ms_per_step": round(float(np.median(step_ms)), 3),
            "host_ms_per_step_call": round(host_s / args.steps * 1e3, 3),
            "p10_p90_ms_per_step": [round(float(np.percentile(step_ms, 10)), 3),
                                    round(float(np.percentile(step_ms, 90)), 3)],
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"{cfg.name} diffusion train step (fwd+bwd+AdamW), "
                                   f"{cfg.image_size[0]}px x{model.n_images} + {model.n_text}-tok text, "
                                   f"ToMe r={cfg.tome_r}/block, {cfg.num_blocks} blocks",
                       "global_batch": N * B, "per_gpu_batch": B, "seq_len": sets0.L,
                       "parallelism": f"dp{N}", "hip_graph": use_graph,
                       "t5_next_step_overlap": t5_pipe,
                       "deterministic": os.environ.get("MMT_DETERMINISTIC", "0") == "1",
                       **({"overrides": over} if over else {}),
                       **({"fp8_weight_path": True} if cfg.fp8 else {})},
            "model_tflops_per_s": round(value * fps / 1e12, 2),
            "algorithmic_gflop_per_sample": round(fps / 1e9, 2),
            "final_loss": round(loss_val, 5),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if di.enabled:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
