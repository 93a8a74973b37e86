"""Host cost of a HIP graph launch: the frozen T5 encoder (B x 32 tokens, OCTO-small's T5-base)
captured (a) on one stream and (b) with one fork / join to a second stream around it, and the
host time of replay() per call (no synchronisation inside the timed loop) against the graph's
kernel count. usage: graph_launch_probe.py [B]"""
import sys
import time

import torch

from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Tokenizer

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
dev = torch.device("cuda:0")
cfg = get_config("octo-small-tome16")
t5 = T5Tokenizer(cfg.t5).materialize(dev, 1)
txt = torch.randint(0, cfg.t5.vocab_size, (B, 32), dtype=torch.int32, device=dev)
out = torch.empty((B, 32, cfg.t5.d_model), dtype=torch.bfloat16, device=dev)


def run_linear():
    out.copy_(t5(txt))


side = torch.cuda.Stream()


def run_forked():
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        out.copy_(t5(txt))
    torch.cuda.current_stream().wait_stream(side)


def many_small(n):
    def f():
        for _ in range(n):
            out.add_(1)
    return f


def probe(name, fn, nodes_hint=""):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    n = 50
    h = 0.0
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        g.replay()
        h += time.perf_counter() - a
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"{name:28s} host {h / n * 1e6:9.1f} us/replay  wall {wall / n * 1e6:9.1f} us/replay {nodes_hint}",
          flush=True)


probe("T5 one stream", run_linear, "(~100 kernels)")
probe("T5 forked to a side stream", run_forked, "(~100 kernels + fork/join)")
probe("200 tiny kernels one stream", many_small(200), "(200 kernels)")
