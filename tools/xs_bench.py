"""Activation-stationary GEMM (csrc/gemm_xs.hip, mmt_gemm_xs) against mmt_gemm's kernels at the
OCTO-small B = 512 short-K shapes: exactness vs the fp32 product (bf16 output rounding), time.
    python tools/xs_bench.py [--b=512]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _C
from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def xs(a, w, out, bias=None):
    M, Kd = a.shape
    N = w.shape[0]
    _C.call("mmt_gemm_xs", M, N, Kd, a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0),
            out.data_ptr(), out.stride(0), None if bias is None else bias.data_ptr(), _C.stream_ptr())


def main():
    dev = torch.device("cuda")
    B = 512
    for a in sys.argv[1:]:
        if a.startswith("--b="):
            B = int(a.split("=")[1])
    torch.manual_seed(0)
    for name, M, N in (("qkv", B * 292, 1152), ("mlp_up", B * 276, 1536), ("small", 1000, 192),
                       ("tail", 777, 1536)):
        Kd = 384
        a = torch.randn((M, Kd), device=dev).bfloat16()
        w = (torch.randn((N, Kd), device=dev) * 0.05).bfloat16()
        bias = torch.randn((N,), device=dev)
        out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        ref = torch.empty_like(out)
        xs(a, w, out, bias)
        K.gemm(a, w, False, True, out=ref, split_k=1, bias=bias)
        torch.cuda.synchronize()
        f32 = (a.float() @ w.float().t() + bias)
        err = ((out.float() - f32).abs().max() / f32.abs().max()).item()
        same = (out == ref).float().mean().item()
        us_x = timeit(lambda: xs(a, w, out, bias))
        us_r = timeit(lambda: K.gemm(a, w, False, True, out=ref, split_k=1, bias=bias))
        fl = 2.0 * M * N * Kd
        by = (M * Kd + M * N) * 2
        print(f"{name:7s} M={M:6d} N={N:5d}: xs {us_x:8.1f} us {fl / us_x / 1e6:7.1f} TF/s {by / us_x / 1e3:6.0f} GB/s | "
              f"mmt_gemm {us_r:8.1f} us {fl / us_r / 1e6:7.1f} TF/s | max rel err vs f32 {err:.2e}, "
              f"bit-equal to mmt_gemm {same * 100:.2f} %", flush=True)
    # the step's MLP up: bias + relu + dropout + relu-bit image, mmt_gemm's dispatch (the
    # activation-stationary kernel) against the 256-wide kernel (variant 5)
    M, N, Kd = B * 276, 1536, 384
    a = torch.randn((M, Kd), device=dev).bfloat16()
    w = (torch.randn((N, Kd), device=dev) * 0.05).bfloat16()
    bias = torch.randn((N,), device=dev)
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    bits = torch.empty((-(-M // 256) * 256, N // 32), dtype=torch.int32, device=dev)
    res = {}
    for v in (-1, 5):
        _C.call("mmt_gemm_set_variant", v)
        try:
            f = lambda: K.gemm(a, w, False, True, out=out, bias=bias, act=K.ACT_RELU, rng=rng,
                               drop_layer=0, drop_site=2, keep_prob=0.9, relu_bits=bits)
            f()
            torch.cuda.synchronize()
            res[v] = (out.clone(), bits.clone(), min(timeit(f) for _ in range(3)))
        finally:
            _C.call("mmt_gemm_set_variant", -1)
    fl = 2.0 * M * N * Kd
    print(f"mlp_up relu+dropout+bits M={M} N={N}: dispatch {res[-1][2]:.1f} us "
          f"({fl / res[-1][2] / 1e6 / 2500:.3f} of peak) | nt256 {res[5][2]:.1f} us "
          f"({fl / res[5][2] / 1e6 / 2500:.3f}) | out equal {torch.equal(res[-1][0], res[5][0])}, "
          f"bits equal {torch.equal(res[-1][1], res[5][1])}", flush=True)


if __name__ == "__main__":
    main()
