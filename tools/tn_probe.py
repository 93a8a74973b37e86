"""Weight-gradient (TN) products of the B = 512 step: libmmt_hip's gemm_tn_dma_kernel (+ split-K
combine) against hipBLASLt (torch.mm on the transposed view, bf16 out, fp32 accumulate) on the
same random operands, graph-timed (tools/gemm_bench.timeit). A known-good reference for what the
chip does on these shapes (cdna_hip_programming.md §5.4 rule 10).

    python tools/tn_probe.py [--b=512] [--wgs=256]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from multi_modal_transformers_tokenmerge_amd.layers import split_k_for
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    B = 512
    wgs = 256
    for a in sys.argv[1:]:
        if a.startswith("--b="):
            B = int(a.split("=")[1])
        if a.startswith("--wgs="):
            wgs = int(a.split("=")[1])
    variants = []
    for a in sys.argv[1:]:
        if a.startswith("--variants="):
            variants = [int(v) for v in a.split("=")[1].split(",")]
    L1, L2 = 292, 276
    if variants:  # libmmt TN kernel variants only, interleaved rounds (mmt_gemm_set_variant)
        from multi_modal_transformers_tokenmerge_amd import _C
        shapes = [("MLP Dense_0 dW", 1536, 384, B * L2), ("MLP Dense_1 dW", 384, 1536, B * L2),
                  ("QKV dW", 1152, 384, B * L1), ("out dW", 384, 384, B * L1)]
        for name, M, N, Kd in shapes:
            dy = (torch.rand((Kd, M), device=dev) * 2 - 1).bfloat16()
            x = (torch.rand((Kd, N), device=dev) * 2 - 1).bfloat16()
            out = torch.zeros((M, N), device=dev, dtype=torch.float32)
            sk = split_k_for(M, N, Kd, wgs=wgs)
            res = {v: [] for v in variants}
            for _ in range(3):
                for v in variants:
                    _C.call("mmt_gemm_set_variant", v)
                    res[v].append(timeit(lambda: K.gemm(dy, x, trans_a=True, out=out,
                                                        out_mode=K.OUT_F32_ACCUM, split_k=sk)))
            _C.call("mmt_gemm_set_variant", -1)
            fl = 2.0 * M * N * Kd
            print(f"{name:16s} {M:5d}x{N:5d}x{Kd:7d} split {sk:3d}: " + "  ".join(
                f"v{v} {min(t):7.1f} us ({fl / min(t) / 2.5e9:.3f})" for v, t in res.items()), flush=True)
        return
    shapes = [("MLP Dense_0 dW", 1536, 384, B * L2), ("MLP Dense_1 dW", 384, 1536, B * L2),
              ("QKV dW", 1152, 384, B * L1), ("out dW", 384, 384, B * L1),
              ("square 4096", 4096, 4096, 4096)]
    for a in sys.argv[1:]:
        if a.startswith("--shapes="):  # e.g. --shapes=0 (the headline dW only, for counter passes)
            shapes = [shapes[int(i)] for i in a.split("=")[1].split(",")]
    for name, M, N, Kd in shapes:
        dy = (torch.rand((Kd, M), device=dev) * 2 - 1).bfloat16()
        x = (torch.rand((Kd, N), device=dev) * 2 - 1).bfloat16()
        out = torch.zeros((M, N), device=dev, dtype=torch.float32)
        sk = split_k_for(M, N, Kd, wgs=wgs)
        t_ours = timeit(lambda: K.gemm(dy, x, trans_a=True, out=out, out_mode=K.OUT_F32_ACCUM, split_k=sk))
        ob = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        t_lib = timeit(lambda: torch.mm(dy.t(), x, out=ob))
        of = torch.empty((M, N), device=dev, dtype=torch.float32)
        try:
            t_lib32 = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=of))
        except Exception as e:  # noqa: BLE001
            t_lib32 = float("nan")
        fl = 2.0 * M * N * Kd
        print(f"{name:16s} {M:5d}x{N:5d}x{Kd:7d} split {sk:3d}: libmmt {t_ours:7.1f} us "
              f"({fl / t_ours / 2.5e9:.3f})  hipBLASLt bf16-out {t_lib:7.1f} us ({fl / t_lib / 2.5e9:.3f})"
              f"  fp32-out {t_lib32:7.1f} us ({fl / t_lib32 / 2.5e9:.3f})", flush=True)


if __name__ == "__main__":
    main()
