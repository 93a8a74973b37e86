"""The frozen T5's products at small batch (M = B * 32 rows): automatic kernel choice vs the
384-wide narrow kernel forced (mmt_gemm_set_variant 8), us per launch by HIP events.
Usage: t5_small_probe.py [M ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _C, _kernels as K

SHAPES = [("qkv", 2304, 768, {}), ("o+res", 768, 768, {"res": True}),
          ("wi relu", 3072, 768, {"act": K.ACT_RELU}), ("wo+res", 768, 3072, {"res": True})]


def time_us(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / n


def split_sweep(dev, Ms):
    """The long-K product with residual (wo 768 x 3072) at split-K 1..4 (auto_split_k's range)."""
    for M in Ms:
        a = torch.randn((M, 3072), device=dev).bfloat16()
        b = torch.randn((768, 3072), device=dev).bfloat16()
        res = torch.randn((M, 768), device=dev).bfloat16()
        ref = None
        for sk in (1, 2, 3, 4):
            out = torch.empty((M, 768), device=dev, dtype=torch.bfloat16)
            t = time_us(lambda: K.gemm(a, b, False, True, out=out, residual=res, split_k=sk))
            d = 0.0 if ref is None else (out.float() - ref).abs().max().item()
            ref = out.float() if ref is None else ref
            print(f"M={M:6d} wo+res split_k={sk}: {t:7.1f} us  max|diff| vs split 1 {d:.3g}", flush=True)


def main():
    dev = torch.device("cuda")
    if sys.argv[1:2] == ["--split"]:
        return split_sweep(dev, [int(x) for x in sys.argv[2:]] or [2048, 4096, 8192])
    for M in [int(x) for x in sys.argv[1:]] or [4096, 8192, 16384]:
        for name, N, Kd, kw in SHAPES:
            a = torch.randn((M, Kd), device=dev).bfloat16()
            b = torch.randn((N, Kd), device=dev).bfloat16()
            res = torch.randn((M, N), device=dev).bfloat16() if kw.get("res") else None
            act = kw.get("act", K.ACT_NONE)
            outs, ts = [], []
            for v in (-1, 8):
                _C.call("mmt_gemm_set_variant", v)
                out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
                ts.append(time_us(lambda: K.gemm(a, b, False, True, out=out, residual=res, act=act, split_k=1)))
                outs.append(out.float())
            _C.call("mmt_gemm_set_variant", -1)
            d = (outs[0] - outs[1]).abs().max().item()
            print(f"M={M:6d} {name:8s} N={N:5d} K={Kd:5d}: auto {ts[0]:7.1f} us  ntw {ts[1]:7.1f} us  "
                  f"max|diff| {d:.3g}", flush=True)


if __name__ == "__main__":
    main()
