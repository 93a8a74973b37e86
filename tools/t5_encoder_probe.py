"""The frozen T5 encoder alone at the bench batch (B x 32 tokens, 12 layers of T5-base), replayed
as a HIP graph: the whole forward's time and, under rocprofv3 --kernel-trace --stats, each of its
kernels standalone (no training step beside it).

    python tools/t5_encoder_probe.py [--b=512] [--reps=20]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo
    B, reps = 512, 20
    for a in sys.argv[1:]:
        if a.startswith("--b="):
            B = int(a.split("=")[1])
        if a.startswith("--reps="):
            reps = int(a.split("=")[1])
    dev = torch.device("cuda")
    model = Octo(get_config("octo-small-tome16"), dev, seed=0)
    txt = torch.randint(0, model.cfg.t5.vocab_size, (B, model.n_text), dtype=torch.int32, device=dev)
    out = torch.empty((B, model.n_text, model.cfg.t5.d_model), dtype=torch.bfloat16, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            out.copy_(model.t5(txt))
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out.copy_(model.t5(txt))
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    e1.synchronize()
    print(f"T5 encoder B={B} ({B * model.n_text} tokens): {e0.elapsed_time(e1) / reps * 1e3:.1f} us per forward")


if __name__ == "__main__":
    main()
