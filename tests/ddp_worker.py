"""One rank of the 2-process data-parallel GPU test (tests/test_ddp_gpu.py); both ranks share the
one GPU and talk over gloo. Not collected by pytest (no test_ prefix).

Checks, on the bench's own step (distributed.DDPStep: staged backward graphs — one per block
here, the "auto" plan with a tiny region target — with each stage's gradient region all-reduced
asynchronously):
  async_vs_sync  : the overlapped all-reduce result equals the one-piece backward + blocking
                   bucketed all-reduce from the same parameters and RNG state;
  shards_vs_full : (rank 0) the all-reduced sum / 2 equals ONE process's gradient of the whole
                   global batch (2 x B samples, sample_offset 0) — per-sample random streams are
                   keyed by the global sample index.
With MMT_DETERMINISTIC=1 (the deterministic mode: fixed-point accumulation at every fp32-atomic
gradient site) also:
  rerun_bitwise  : the staged step run twice gives the same all-reduced gradients bit for bit;
  tome_equal     : this rank's ToMe index triples equal, bit for bit, its rows of the full global
                   batch's triples at every merging layer.
Writes a JSON report to argv[1].
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rel_by_tensor(model, a, b):
    worst = 0.0
    for p in model.store.params:
        x = a[p.offset:p.offset + p.numel].double()
        y = b[p.offset:p.offset + p.numel].double()
        n = float(y.norm())
        if n > 0:
            worst = max(worst, float((x - y).norm()) / n)
    return worst


def main():
    out_path = sys.argv[1]
    from multi_modal_transformers_tokenmerge_amd.distributed import DDPStep, GradAllReducer, init_from_env
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    from oracle.parity import _inputs
    di = init_from_env(backend="gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, N = 2, di.world_size
    cfg = get_config("octo-tiny", num_blocks=4, token_compression_sequence="[Image{2};Readout{0}]")
    model = Octo(cfg, dev, seed=0)
    images, _, actions = _inputs(model, N * B, seed=3)        # the global batch
    img_all = torch.from_numpy(images).to(dev)
    act_all = torch.from_numpy(actions).to(dev)
    sl = slice(di.rank * B, (di.rank + 1) * B)
    img, act = img_all[sl].contiguous(), act_all[sl].contiguous()
    red = GradAllReducer(N, bucket_bytes=1 << 20)
    state = create_octo_train_state(model, seed=11, allreduce=red, sample_offset=di.rank * B)
    # the bench's default plan ("auto": byte-sized gradient regions, block 0 alone last); a tiny
    # region target gives every block its own stage and region here
    step = DDPStep(model, state, None, img, act, red, stages="auto:0.001", use_graph=True).build(warm=1)
    assert step.bounds == [4, 3, 2, 1, 0], step.bounds
    step()                                   # a real step, then freeze params + RNG
    torch.cuda.synchronize()
    P = model.store.flat.clone()
    rng0 = state.rng.clone()

    def restore():
        model.store.flat.copy_(P)
        model.store.sync_shadow()
        state.rng.copy_(rng0)
        torch.cuda.synchronize()

    restore()
    step()                                   # staged graphs + async region all-reduces
    torch.cuda.synchronize()
    g_async = model.store.flat_grad.clone()
    restore()
    model.store.zero_grad()
    _, st = model.compute_diffusion_denoise_loss(None, img, act, True, state.rng, state.sample_offset)
    model.backward(st)
    red(model.store.flat_grad)               # blocking bucketed all-reduce
    torch.cuda.synchronize()
    g_sync = model.store.flat_grad.clone()
    rep = dict(rank=di.rank, async_vs_sync=rel_by_tensor(model, g_async, g_sync),
               stages=step.S, exposed_bytes=step.exposed_bytes)
    if os.environ.get("MMT_DETERMINISTIC", "0") == "1":
        restore()
        step()
        torch.cuda.synchronize()
        rep["rerun_bitwise"] = bool(torch.equal(model.store.flat_grad, g_async))
        restore()
        _, st = model.compute_diffusion_denoise_loss(None, img, act, True, state.rng, state.sample_offset)
        mine = [sv["tome"][6:9] for sv in st["stack_sv"] if sv["tome"] is not None]
        restore()
        _, st = model.compute_diffusion_denoise_loss(None, img_all, act_all, True, state.rng, 0)
        full = [sv["tome"][6:9] for sv in st["stack_sv"] if sv["tome"] is not None]
        rep["tome_layers"] = len(mine)
        rep["tome_equal"] = len(mine) == len(full) and all(
            torch.equal(a, b[sl]) for m, f in zip(mine, full) for a, b in zip(m, f))
        torch.cuda.synchronize()
    dist.barrier()
    if di.rank == 0:
        restore()
        model.store.zero_grad()
        _, st = model.compute_diffusion_denoise_loss(None, img_all, act_all, True, state.rng, 0)
        model.backward(st)
        torch.cuda.synchronize()
        rep["shards_vs_full"] = rel_by_tensor(model, g_sync / N, model.store.flat_grad)
        rep["grad_norm"] = float(g_sync.norm())
    dist.barrier()
    dist.destroy_process_group()
    with open(out_path, "w") as fh:
        json.dump(rep, fh)
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
