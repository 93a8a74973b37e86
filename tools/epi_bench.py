"""Epilogue cost ablation of the wide nt256 GEMM at the OCTO-small MLP shapes (B = 256):
the MLP-up product with each epilogue feature on its own and all together, and the gated MLP dX
product (relu gate, dropout mask, column sums). HIP-event timed over graph replays."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    M = 256 * 276
    cases = [
        ("up plain", 1536, 384, {}),
        ("up bias", 1536, 384, dict(bias="f32")),
        ("up relu", 1536, 384, dict(act=K.ACT_RELU)),
        ("up drop", 1536, 384, dict(rng=rng, keep_prob=0.9)),
        ("up bias+relu+drop", 1536, 384, dict(bias="f32", act=K.ACT_RELU, rng=rng, keep_prob=0.9)),
        ("dX plain", 1536, 384, {}),
        ("dX gate", 1536, 384, dict(gate="bf16")),
        ("dX gate+drop", 1536, 384, dict(gate="bf16", rng=rng, keep_prob=0.9)),
        ("dX gate+drop+colsum", 1536, 384, dict(gate="bf16", rng=rng, keep_prob=0.9, colsum=True)),
        ("qkv plain", 1152, 384, {}),
        ("qkv bias", 1152, 384, dict(bias="f32")),
        ("down f32 plain", 384, 1536, dict(out=K.OUT_F32)),
        ("down f32 bias+drop+res", 384, 1536, dict(out=K.OUT_F32, bias="f32", rng=rng, keep_prob=0.9,
                                                   residual="f32")),
        ("dX384 bf16 plain", 384, 1536, {}),
        ("oproj f32 bias+drop+res", 384, 384, dict(out=K.OUT_F32, bias="f32", rng=rng, keep_prob=0.9,
                                                   residual="f32")),
        ("dX384k384 bf16 plain", 384, 384, {}),
        ("dX384k1152 bf16 plain", 384, 1152, {}),
    ]
    only = [a for a in sys.argv[1:] if not a.startswith("-")]
    for name, N, Kd, epi in cases:
        if only and not any(o in name for o in only):
            continue
        a = torch.randn((M, Kd), device=dev).bfloat16()
        b = torch.randn((N, Kd), device=dev).bfloat16()
        e = dict(epi)
        if e.get("bias") == "f32":
            e["bias"] = torch.randn(N, device=dev)
        if e.get("gate") == "bf16":
            e["gate"] = torch.randn((M, N), device=dev).bfloat16()
        if e.get("colsum"):
            rows = K.gemm_colsum_rows(M, N, Kd)
            e["colsum"] = torch.zeros((rows, N), device=dev)
        if e.get("residual") == "f32":
            e["residual"] = torch.randn((M, N), device=dev)
        om = e.pop("out", K.OUT_BF16)
        out = torch.empty((M, N), device=dev, dtype=torch.bfloat16 if om == K.OUT_BF16 else torch.float32)
        us = timeit(lambda: K.gemm(a, b, False, True, out=out, out_mode=om, split_k=1, **e))
        print(f"{name:24s} M={M} N={N} K={Kd}: {us:8.1f} us  {2 * M * N * Kd / us / 1e6:7.1f} TF/s",
              flush=True)


if __name__ == "__main__":
    main()
