#!/usr/bin/env python3
"""Benchmark of the hot path: train samples/sec of the OCTO-small diffusion training step
(256x256 image + 32-token text, ToMe r=16 per block, bf16 MFMA) on N MI355X — BASELINE.json's
metric, config[2] (the single-GPU line uses the same workload at N=1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--config NAME]
    torchrun --nproc-per-node N bench.py --gpus N ...          (one process per GPU, RCCL)

Per-GPU batch 256 by default (measured 5.7k / 7.4k / 8.6k / 9.1k samples/s at B = 64 / 128 / 256 /
512 on one MI355X: at B = 64 the launches are too small to fill 256 CUs; see DESIGN.md "Batch").
One step = zero grads -> forward (frozen T5, image stem, 12 ToMe blocks, diffusion loss) ->
backward -> [gradient all-reduce over RCCL] -> fused AdamW -> device step counter, on synthetic
inputs resident in HBM (numpy default_rng(0) shapes of SURVEY §8d). The N=1 step is one HIP graph
replay; with N>1 the backward runs as --overlap-stages block-range graphs, each stage's gradient
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
    for (sets, _, ts, r, prune) in model.layer_sets:
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


PROBE_KERNEL = "gemm_nt256_kernel<256, 0, false, 2>"


def probe_dominant_gemm(model, B, reps=20):
    """Average duration (HIP events on the launching stream) of the MLP up-projection GEMM of
    block 0 at the step's exact shape: M = B*L1, N = mlp_dim, K = D (bias+relu+dropout fused);
    the library's automatic choice for this NT shape (N >= 1152, N % 256 == 0, K <= 512) is the
    persistent 256 x 256 kernel gemm_nt256_kernel<256, 0, false, 2> (csrc/gemm.hip)."""
    cfg = model.cfg
    blk = model.stack.blocks[0]
    sets, _, ts, r, prune = model.layer_sets[0]
    M = B * (sum(prune[1]) if prune else sets.L - r)
    D = cfg.token_embedding_dim
    x = torch.randn((M, D), device=model.device).to(torch.bfloat16)
    rng = torch.tensor([7, 1], dtype=torch.int32, device=model.device)
    out = torch.empty((M, cfg.mlp_dim), dtype=torch.bfloat16, device=model.device)

    def launch():
        blk.mlp.dense.fwd(x, out=out, act=K.ACT_RELU, rng=rng, drop_layer=0, drop_site=2,
                          keep_prob=0.9)
    # reps launches captured in one HIP graph (as in the training step: no host launch gaps),
    # timed with HIP events recorded on the stream the graph replays on
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
    avg_ms = e0.elapsed_time(e1) / reps
    flops = 2.0 * M * cfg.mlp_dim * D
    return dict(kernel=PROBE_KERNEL + " (MLP Dense_0 fwd, bias+relu+dropout epilogue)",
                shape=[M, cfg.mlp_dim, D], avg_us=avg_ms * 1e3, flops=flops,
                tflops=flops / (avg_ms * 1e-3) / 1e12)


def gemm_traffic(shape):
    """HBM bytes per launch of the probe GEMM from the committed rocprofv3 PMC passes
    (profiles/*_gemm_pmc.json, written by tools/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE,
    the gfx950 correction of MI355X_MICROARCH.md "HBM"), or None when no pass matches."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_gemm_pmc.json")), reverse=True):
        with open(f) as fh:
            d = json.load(fh)
        if list(d.get("shape_MNK", [])) == list(shape) and d.get("kernel") == PROBE_KERNEL:
            return d["hbm_bytes_per_launch"]
    return None


def cpu_baseline(cfg_name, model, budget_s=15.0, B=2):
    """fp32 CPU restatement (oracle/octo_ref.py) forward+backward+AdamW on a bounded sample."""
    from oracle.octo_ref import OctoRef, sequence_spec
    cfg = model.cfg
    threads = torch.get_num_threads()
    params = {p.name: p.data.detach().float().cpu().clone().requires_grad_() for p in model.store.params}
    t5p = ({p.name: p.bf16.float().cpu() for p in model.t5.store.params} if model.has_text else None)
    ref = OctoRef(cfg, params, t5p)
    opt = torch.optim.AdamW(list(params.values()), lr=3e-4, weight_decay=1e-4)
    g = np.random.default_rng(0)
    H = cfg.image_size[0]
    images = g.integers(0, 256, (B, model.n_images, H, H, 3)).astype(np.float32)
    text = g.integers(0, cfg.t5.vocab_size, (B, model.n_text)).astype(np.int32) if model.has_text else None
    actions = g.uniform(-1, 1, (B, cfg.action_space_dim)).astype(np.float32)
    npat = model.image_tokenizer.num_patches * model.n_images
    pos = (g.integers(0, 127, (B, npat)), g.integers(0, 127, (B, npat)))
    spec = sequence_spec(cfg.input_sequence, cfg.token_compression_sequence)

    def step(i):
        opt.zero_grad(set_to_none=True)
        loss, _ = ref.forward_loss(text, images, actions, seed=1, step=i, positions=pos,
                                   t=g.integers(0, cfg.diffusion_steps, B),
                                   eps=g.standard_normal((B, cfg.action_space_dim)).astype(np.float32),
                                   sequence=spec)
        loss.backward()
        opt.step()
    step(0)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step(n + 1)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 50:
            break
    return dict(value=B * n / el, unit="samples/s", cores=threads, kind="port",
                sample=f"{cfg_name} fp32 torch-CPU restatement (oracle/octo_ref.py), per-step fwd+bwd+AdamW, "
                       f"B={B}, {n} timed steps in {el:.1f}s after 1 warm-up "
                       "(JAX reference not importable offline)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256,
                    help="per-GPU batch (256: see DESIGN.md 'Batch'; 64 leaves the chip underfilled)")
    ap.add_argument("--config", default="octo-small-tome16")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--overlap-stages", type=int, default=3,
                    help="N > 1: backward split into this many block ranges, each range's gradient "
                         "all-reduce overlapped with the rest of the backward (1 = no overlap)")
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
    cfg = get_config(args.config)
    B = args.batch
    model = Octo(cfg, dev, seed=0)
    if args.probe_only:
        probe = probe_dominant_gemm(model, B, reps=50)
        print(json.dumps(dict(probe_only=True, **probe)), flush=True)
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
    step = DDPStep(model, state, txt, img, act, reducer, stages=args.overlap_stages,
                   use_graph=use_graph).build()
    loss_buf = step.loss_buf

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if di.enabled:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if di.enabled:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if di.enabled:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss_val = float(loss_buf.item())

    if di.rank == 0:
        ms = elapsed / args.steps * 1e3
        value = N * B * args.steps / elapsed
        probe = probe_dominant_gemm(model, B)
        roof = dict(bound="mfma", achieved=round(probe["tflops"], 2), peak=MFMA_BF16_PEAK_TFLOPS,
                    unit="TFLOP/s", frac=round(probe["tflops"] / MFMA_BF16_PEAK_TFLOPS, 4),
                    traffic=gemm_traffic(probe["shape"]), kernel=probe["kernel"], shape_MNK=probe["shape"],
                    avg_launch_us=round(probe["avg_us"], 2),
                    flops_per_launch=probe["flops"],
                    algorithmic_bytes_per_launch=2 * (probe["shape"][0] * probe["shape"][2]
                                                      + probe["shape"][1] * probe["shape"][2]
                                                      + probe["shape"][0] * probe["shape"][1])
                    + 4 * probe["shape"][1])
        fps = algorithmic_flops_per_sample(model)
        cpu = None
        if N == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.config, model, budget_s=args.cpu_budget)
        sets0 = model.layer_sets[0][0]
        line = {
            "metric": "train samples/sec OCTO-small 256px+text, ToMe r=16, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "samples/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"{cfg.name} diffusion train step (fwd+bwd+AdamW), "
                                   f"{cfg.image_size[0]}px x{model.n_images} + {model.n_text}-tok text, "
                                   f"ToMe r={cfg.tome_r}/block, {cfg.num_blocks} blocks",
                       "global_batch": N * B, "per_gpu_batch": B, "seq_len": sets0.L,
                       "parallelism": f"dp{N}", "hip_graph": use_graph},
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
