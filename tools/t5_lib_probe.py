"""The frozen T5 encoder's four products at B = 512 (M = 16,384 tokens, d_model 768, d_ff 3072):
libmmt_hip's kernels (what the step runs) against hipBLASLt on the same operands, graph-timed.

    python tools/t5_lib_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    M = 16384
    for a in sys.argv[1:]:
        if a.startswith("--m="):
            M = int(a.split("=")[1])
    g = torch.Generator(device="cpu").manual_seed(0)
    def mk(*s):
        return (torch.randn(s, generator=g) * 0.05).bfloat16().to(dev)
    x768, h3072 = mk(M, 768), mk(M, 3072)
    wqkv, wo, wi, wo2 = mk(2304, 768), mk(768, 768), mk(3072, 768), mk(768, 3072)
    res = mk(M, 768)
    z3072 = torch.zeros(3072, dtype=torch.bfloat16, device=dev)
    cases = [
        ("qkv 16384x2304x768", lambda: K.gemm(x768, wqkv, trans_b=True), lambda: torch.mm(x768, wqkv.t()), 2 * M * 2304 * 768),
        ("o + residual 768x768", lambda: K.gemm(x768, wo, trans_b=True, residual=res),
         lambda: torch.addmm(res, x768, wo.t()), 2 * M * 768 * 768),
        ("ff in relu 3072x768", lambda: K.gemm(x768, wi, trans_b=True, act=K.ACT_RELU),
         lambda: torch._addmm_activation(z3072, x768, wi.t()), 2 * M * 3072 * 768),
        ("ff out + residual 768x3072", lambda: K.gemm(h3072, wo2, trans_b=True, residual=res),
         lambda: torch.addmm(res, h3072, wo2.t()), 2 * M * 768 * 3072),
    ]
    for name, ours, lib, fl in cases:
        a = [timeit(ours), timeit(lib), timeit(ours), timeit(lib)]
        to, tl = min(a[0], a[2]), min(a[1], a[3])
        print(f"M={M} {name:28s} libmmt {to:7.1f} us ({fl / to / 2.5e9:.3f})  hipBLASLt {tl:7.1f} us "
              f"({fl / tl / 2.5e9:.3f})", flush=True)


if __name__ == "__main__":
    main()
