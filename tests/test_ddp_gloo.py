"""Data-parallel logic on CPU: world_size 2 over gloo (127.0.0.1), one process per rank.

Covers distributed.init_from_env (torchrun env contract), the bucketed flat-gradient all-reduce
with the 1/N average folded into grad_scale, the rank-0 parameter broadcast, and the max-over-ranks
timing reduction bench.py uses.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from multi_modal_transformers_tokenmerge_amd.distributed import GradAllReducer, init_from_env
    try:
        di = init_from_env(backend="gloo")
        assert di.enabled and di.rank == rank and di.world_size == world
        n = 10_007                                  # not a multiple of the bucket size
        grad = (rank + 1) * torch.arange(n, dtype=torch.float32)
        red = GradAllReducer(world, bucket_bytes=4 * 1000)
        red(grad)
        expect = sum(r + 1 for r in range(world)) * torch.arange(n, dtype=torch.float32)
        ok_sum = bool(torch.equal(grad, expect))
        ok_scale = red.grad_scale == 1.0 / world
        params = torch.full((17,), float(rank))
        dist.broadcast(params, 0)
        ok_bcast = bool((params == 0).all())
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ok_max = float(t.item()) == world
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ok_sum, ok_scale, ok_bcast, ok_max))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.timeout(120)
def test_gloo_world2_allreduce_broadcast():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert len(r) == 5 and all(r[1:]), r


def test_single_process_is_not_distributed(monkeypatch):
    from multi_modal_transformers_tokenmerge_amd.distributed import GradAllReducer, init_from_env
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    di = init_from_env()
    assert not di.enabled and di.rank == 0
    g = torch.ones(5)
    GradAllReducer(1)(g)                          # no-op without a process group
    assert torch.equal(g, torch.ones(5))
