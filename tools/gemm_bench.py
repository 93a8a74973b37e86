"""Micro-benchmark of libmmt_hip's MFMA GEMM at the OCTO-small training-step shapes (B=64).
Times each variant with HIP events on the launching stream; prints TFLOP/s."""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K


def timeit(fn, reps=20):
    """Average kernel time of fn: reps launches captured in one HIP graph and replayed, so host
    launch overhead (Python + ctypes, ~10 us per call) is excluded, as in the training step."""
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
    cur = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(cur)
    for _ in range(3):
        g.replay()
    b.record(cur)
    b.synchronize()
    return a.elapsed_time(b) / (3 * reps) * 1e3  # us


def main():
    from multi_modal_transformers_tokenmerge_amd import _C
    for a in sys.argv[1:]:
        if a.startswith("--variant="):
            _C.call("mmt_gemm_set_variant", int(a.split("=")[1]))
            print("variant", a, flush=True)
    dev = torch.device("cuda")
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    if "--sweep" in sys.argv:  # fixed cost vs per-K-step cost of one launch shape
        for (M, N) in [(18688, 384), (18688, 1536)]:
            for Kd in [64, 128, 256, 384, 768, 1536]:
                a = torch.randn((M, Kd), device=dev).bfloat16()
                b = torch.randn((N, Kd), device=dev).bfloat16()
                out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
                us = timeit(lambda: K.gemm(a, b, False, True, out=out, split_k=1))
                print(f"sweep M={M} N={N} K={Kd:5d}: {us:8.2f} us  {2*M*N*Kd/us/1e6:7.1f} TF/s", flush=True)
        return
    Bsz = 256
    for a in sys.argv[1:]:
        if a.startswith("--b="):
            Bsz = int(a.split("=")[1])
    M1 = Bsz * 276
    cases = []
    # (name, M, N, K, ta, tb, out_mode, epi)
    for (M, N, Kd) in [(M1, 1536, 384), (M1, 384, 1536), (Bsz * 292, 1152, 384), (Bsz * 292, 384, 384), (Bsz * 32, 768, 3072), (Bsz * 32, 2304, 768),
                       (4096, 4096, 4096)]:
        cases.append(("fwd NT plain", M, N, Kd, False, True, K.OUT_BF16, {}))
    cases.append(("fwd NT bias+relu+drop", M1, 1536, 384, False, True, K.OUT_BF16,
                  dict(act=K.ACT_RELU, rng=rng, keep_prob=0.9)))
    cases.append(("fwd NT f32 out + residual f32 + drop", M1, 384, 1536, False, True, K.OUT_F32,
                  dict(rng=rng, keep_prob=0.9, residual="f32")))
    cases.append(("dX NN plain", M1, 384, 1536, False, False, K.OUT_BF16, {}))
    cases.append(("dX NN gate", M1, 1536, 384, False, False, K.OUT_BF16, dict(gate="bf16")))
    cases.append(("dX NN f32", M1, 384, 1536, False, False, K.OUT_F32, {}))
    cases.append(("dW TN splitK", 1536, 384, M1, True, False, K.OUT_F32_ACCUM, {}))
    cases.append(("dW TN splitK", 384, 1536, M1, True, False, K.OUT_F32_ACCUM, {}))
    cases.append(("dW TN splitK", 1152, 384, Bsz * 292, True, False, K.OUT_F32_ACCUM, {}))
    for name, M, N, Kd, ta, tb, om, epi in cases:
        a = torch.randn((Kd, M) if ta else (M, Kd), device=dev).bfloat16()
        b = torch.randn((N, Kd) if tb else (Kd, N), device=dev).bfloat16()
        e = dict(epi)
        if e.get("residual") == "f32":
            e["residual"] = torch.randn((M, N), device=dev)
        if e.get("gate") == "bf16":
            e["gate"] = torch.randn((M, N), device=dev).bfloat16()
        out = torch.zeros((M, N), device=dev, dtype=torch.bfloat16 if om == K.OUT_BF16 else torch.float32)
        sk = 1
        if om == K.OUT_F32_ACCUM:
            from multi_modal_transformers_tokenmerge_amd.layers import split_k_for
            sk = split_k_for(M, N, Kd)
        us = timeit(lambda: K.gemm(a, b, ta, tb, out=out, out_mode=om, split_k=sk, **e))
        print(f"{name:40s} M={M:6d} N={N:5d} K={Kd:6d} split={sk:2d}: {us:8.1f} us  {2*M*N*Kd/us/1e6:7.1f} TF/s", flush=True)
    # library reference point (hipBLASLt through torch.matmul), plain bf16 output, same shapes
    if "--torch" in sys.argv:
        for (M, N, Kd, ta, tb) in [(M1, 1536, 384, False, True), (M1, 384, 1536, False, True),
                                   (Bsz * 292, 1152, 384, False, True), (Bsz * 32, 768, 3072, False, True),
                                   (M1, 384, 1536, False, False), (1536, 384, M1, True, False),
                                   (4096, 4096, 4096, False, True)]:
            a = torch.randn((Kd, M) if ta else (M, Kd), device=dev).bfloat16()
            b = torch.randn((N, Kd) if tb else (Kd, N), device=dev).bfloat16()
            A = a.t() if ta else a
            Bm = b.t() if tb else b
            us = timeit(lambda: torch.matmul(A, Bm))
            print(f"torch.matmul ta={ta:d} tb={tb:d}               M={M:6d} N={N:5d} K={Kd:6d}         : {us:8.1f} us  {2*M*N*Kd/us/1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
