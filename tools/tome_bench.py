"""ToMe kernels in isolation (at B >= 256 a per-layer launch is not launch-bound).

Shapes of OCTO-small block 0: sequence L = 292 (32 text + 256 image + 4 readouts), image set at
rows [32, 288), t = 256, r = 16, D = 384 fp32 residual stream, metric = sum over 6 heads of the
bf16 K projection read in place from the (B, L, 3*384) QKV buffer.

Algorithmic HBM bytes per sample (§8d, with this build's dtypes):
  match     t*H*c*2 (bf16 K heads) + 4*(ceil(t/2) + 2r) (indices)
  merge fwd t*D*4 + t*4 + (t-r)*D*4 + (t-r)*4   (+ the 36 copied non-set rows: 2*36*D*4)
  merge bwd the same with read and write swapped
Times: launches captured in a HIP graph and replayed (no host launch gaps).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K

HBM_GBS = 8000.0


def graph_time(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    a.record(cur)
    for _ in range(3):
        g.replay()
    b.record(cur)
    b.synchronize()
    return a.elapsed_time(b) / (3 * reps) * 1e3


def main():
    dev = torch.device("cuda")
    out = []
    shapes = [(n, 292, 32, 256, 16, 384, 6, 64) for n in (64, 256, 512)] + \
        [(n, 1060, 32, 1024, 32, 768, 12, 64) for n in (16, 64)]      # OCTO-base hi-res block 0
    for n, L, s0, t, r, D, H, c in shapes:
        g = torch.Generator(device="cpu").manual_seed(n)
        qkv = torch.randn((n, L, 3 * D), generator=g).bfloat16().to(dev)
        metric = qkv[:, s0:s0 + t, D:2 * D].view(n, t, H, c)     # strided K heads, in place
        x = torch.randn((n, L, D), generator=g).to(dev)
        size = torch.rand((n, t), generator=g).add_(1).to(dev)
        unm, src, dst = K.tome_match(metric, r)
        xo, so, pm = K.tome_merge_fwd(x, s0, t, r, unm, src, dst, size_in=size)
        gout = torch.randn_like(xo)
        us_m = graph_time(lambda: K.tome_match(metric, r))
        us_f = graph_time(lambda: K.tome_merge_fwd(x, s0, t, r, unm, src, dst, size_in=size, out=xo))
        us_b = graph_time(lambda: K.tome_merge_bwd(gout, s0, t, r, pm, size, so))
        ta = (t + 1) // 2
        b_match = n * (t * H * c * 2 + 4 * (ta + 2 * r))
        b_set = n * (t * D * 4 + t * 4 + (t - r) * D * 4 + (t - r) * 4)
        b_all = b_set + n * 2 * (L - t) * D * 4
        for name, us, byts in (("match", us_m, b_match), ("merge_fwd", us_f, b_all),
                               ("merge_bwd", us_b, b_all)):
            gbs = byts / us / 1e3
            out.append(dict(kernel=name, n=n, t=t, us=round(us, 2), bytes=byts, GBps=round(gbs, 1),
                            hbm_frac=round(gbs / HBM_GBS, 3),
                            set_only_GBps=round((b_set if name != "match" else b_match) / us / 1e3, 1)))
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
