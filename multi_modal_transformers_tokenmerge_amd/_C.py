"""ctypes binding of libmmt_hip.so (the C ABI declared in include/mmt_api.h).

There is deliberately no CPU or PyTorch fallback: if the library is missing every op raises.
Build it with ``python -m multi_modal_transformers_tokenmerge_amd.csrc.build`` (or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
from pathlib import Path

_LIB_PATH = Path(__file__).resolve().parent / "libmmt_hip.so"
_lib = None

P, I, L, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
U32, U64, Z = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
D = ctypes.c_double

class Epilogue(ctypes.Structure):
    """mmt_epilogue_t (include/mmt_api.h)."""
    _fields_ = [("bias", P), ("act", I), ("rng", P), ("drop_layer", U32), ("drop_site", U32),
                ("keep_prob", F), ("drop_row_offset", L), ("gate", P), ("ld_gate", L),
                ("gate_scale", F), ("residual", P), ("ld_res", L), ("alpha", F), ("beta", F),
                ("res_dtype", I), ("colsum", P), ("relu_bits", P), ("gate_bits", P),
                ("keep_bits", P)]


# name -> argtypes (every entry point returns int status unless listed in _VOID)
SIGNATURES: dict[str, list] = {
    "mmt_version": [],
    "mmt_device_status": [P],
    "mmt_tome_set_match_path": [I],
    "mmt_workspace_size": [I, P, I],
    "mmt_tome_match": [P, I, I, I, I, I, L, L, L, I, I, P, P, P, P, P, L, P],
    "mmt_tome_merge_wavg_fwd": [P, I, I, I, I, L, L, I, I, I, I, P, P, P, P, P, L, L, P, P, P],
    "mmt_tome_merge_wavg_bwd": [P, I, I, I, I, L, L, I, I, I, P, P, P, P, L, L, P],
    "mmt_seqnorm_dropout_bwd": [P, L, L, P, L, L, I, I, I, P, P, P, P, L, L, P, L, L, P, P, P, U32,
                                U32, F, L, P, L, L, P, P],
    "mmt_ln_unmerge_dropout_bwd": [P, L, L, P, L, L, I, I, I, P, P, P, P, L, L, P, P, I, I, I, I, P,
                                   P, P, P, L, L, P, U32, U32, F, L, P, L, L, P, P],
    "mmt_tome_merge_seqnorm_fwd": [P, I, I, I, L, L, I, I, I, I, P, P, P, P, P, L, L, P, P, P, P, F,
                                   P, L, L, P, P, P],
    "mmt_topk_gather": [P, I, I, I, I, L, L, P, L, I, P, P, P, P, L, L, P, P],
    "mmt_topk_scatter_bwd": [P, I, I, I, I, L, L, P, I, P, L, L, P],
    "mmt_gemm_set_variant": [I],
    "mmt_set_deterministic": [P, P, L],
    "mmt_det_flush": [P, P, L, P],
    "mmt_gemm_colsum_rows": [I, I, I, I, I, I, I],
    "mmt_gemm_dropout_keep_bits": [P, U32, U32, I, I, F, L, P, P],
    "mmt_gemm": [I, I, I, P, I, L, P, I, L, P, I, L, I, L, L, L, I, P, P, L, P],
    "mmt_quant_rows_fp8": [P, L, I, I, P, L, P, P],
    "mmt_gemm_fp8": [I, I, I, P, L, P, P, L, P, P, I, L, P, P],
    "mmt_gemm_xs": [I, I, I, P, L, P, L, P, L, P, P],
    "mmt_attn_fwd": [P, L, L, I, I, I, I, F, I, P, P, P, P, F, P, P, L, L, P, P, P],
    "mmt_prune_importance": [P, I, I, I, P, P],
    "mmt_gather_rows": [P, I, I, I, I, L, L, P, I, P, L, L, P],
    "mmt_maxpool2d": [P, L, I, I, I, I, P, P, P],
    "mmt_maxpool2d_bwd": [P, P, L, I, I, I, I, P, P],
    "mmt_im2col_same": [P, L, I, I, I, I, P, P],
    "mmt_col2im_same": [P, L, I, I, I, I, P, P],
    "mmt_attn_bwd": [P, L, L, I, I, I, I, F, I, P, P, P, P, P, F, P, L, L, P, L, L, P, P, P, L, L, P, P],
    "mmt_dropout_bits": [P, U32, U32, I, I, F, P, P, P],
    "mmt_seqnorm_fwd": [P, I, L, L, I, I, I, P, P, F, P, L, L, P, P, P],
    "mmt_seqnorm_bwd": [P, I, L, L, P, I, L, L, I, I, I, P, P, P, P, L, L, P, L, L, P, P, P],
    "mmt_colsum": [P, I, L, I, I, P, P],
    "mmt_dropout_bwd": [P, I, L, I, I, P, U32, U32, F, L, P, L, P, P],
    "mmt_patch_im2col": [P, I, I, I, I, I, I, I, I, I, I, P, P],
    "mmt_maxpool_patch": [P, L, I, I, P, P, P],
    "mmt_maxpool_patch_bwd": [P, P, L, I, I, P, P],
    "mmt_groupnorm_gelu_fwd": [P, I, I, I, I, F, P, P, P, P, P, P],
    "mmt_groupnorm_gelu_bwd": [P, P, I, I, I, I, P, P, P, P, P, I, P, P, P],
    "mmt_patch_positions": [P, U32, I, I, I, I, I, I, L, P, P, P],
    "mmt_seq_assemble_fwd": [I, I, I, P, P, I, P, I, P, P, P, P, P, P, P, P],
    "mmt_seq_assemble_bwd": [I, I, I, P, P, P, I, P, I, P, P, P, I, P, P, P, P],
    "mmt_patch_embed_grad": [I, I, I, I, I, I, I, P, P, P, P, P, P, P],
    "mmt_stem_conv_pool": [P, I, I, I, P, P, P, P, P],
    "mmt_stem_conv_wgrad_slabs": [I, I, I],
    "mmt_stem_conv_wgrad": [P, I, I, I, P, P, P, L, P],
    "mmt_add_position_embedding": [P, P, P, I, I, I, P],
    "mmt_rows_mean_fwd": [P, L, L, I, I, P, I, P, L, P],
    "mmt_rows_mean_bwd": [P, L, I, I, I, P, I, P, P],
    "mmt_diffusion_prep": [P, I, I, I, L, P, P, P, I, P, P, P, P, P, L, P, P],
    "mmt_fourier_bwd": [P, I, I, P, P, P, P],
    "mmt_diffusion_loss": [P, L, P, I, I, F, P, P, P],
    "mmt_diffusion_sample": [P, I, I, I, L, P, L, P, L, P, L, P, P, P, P, I, P, P, P],
    "mmt_rows_group_mean_fwd": [P, L, L, I, I, I, P, I, P, P, P],
    "mmt_rows_group_mean_bwd": [P, I, I, I, P, I, P, P, P],
    "mmt_action_head": [I, P, L, I, I, P, P, I, F, F, P, P, P, P],
    "mmt_rmsnorm_fwd": [P, L, I, P, F, P, P],
    "mmt_embedding_gather": [P, L, I, P, I, P, P],
    "mmt_adamw": [P, P, P, P, P, L, P, D, D, D, D, D, F, P],
    "mmt_cast_f32_bf16": [P, P, L, P],
    "mmt_transpose_bf16_batched": [P, P, P, I, L, P],
    "mmt_step_advance": [P, P],
}
_VOID = {"mmt_tome_set_match_path", "mmt_gemm_set_variant"}
_RESTYPE = {"mmt_workspace_size": L,      # returns a byte count (negative: error)
            "mmt_gemm_colsum_rows": I,    # returns a row count
            "mmt_stem_conv_wgrad_slabs": I}


API_VERSION = 2  # include/mmt_api.h MMT_API_VERSION


class MMTError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            raise ImportError(f"{_LIB_PATH} is missing: build it with "
                              "`python -m multi_modal_transformers_tokenmerge_amd.csrc.build` "
                              "(no CPU fallback exists by design)")
        import os
        import sys
        path = str(_LIB_PATH)
        ab = os.environ.get("MMT_LIB_AB")
        if ab:  # benchmarking knob: A/B a second build of the same C ABI from inside the build tree
            p = Path(ab).resolve()
            root = _LIB_PATH.resolve().parent.parent
            if root not in p.parents or p.suffix != ".so":
                raise ImportError(f"MMT_LIB_AB={ab!r}: only a .so inside {root} may replace "
                                  f"{_LIB_PATH.name}")
            print(f"[mmt] MMT_LIB_AB: loading {p} instead of {_LIB_PATH}", file=sys.stderr)
            path = str(p)
        h = ctypes.CDLL(path)
        h.mmt_last_error.restype = ctypes.c_char_p
        h.mmt_last_error.argtypes = []
        for name, args in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = None if name in _VOID else _RESTYPE.get(name, I)
        if h.mmt_version() != API_VERSION:  # the Epilogue layout above is version 2's
            raise ImportError(f"{path}: C ABI version {h.mmt_version()}, this binding needs "
                              f"{API_VERSION} (include/mmt_api.h MMT_API_VERSION): rebuild it")
        _lib = h
        if os.environ.get("MMT_GEMM_VARIANT"):  # benchmarking knob (include/mmt_api.h)
            h.mmt_gemm_set_variant(int(os.environ["MMT_GEMM_VARIANT"]))
    return _lib


def call(name: str, *args) -> int:
    rc = getattr(lib(), name)(*args)
    if name in _VOID:
        return 0
    if name in _RESTYPE:
        if rc < 0:
            raise MMTError(f"{name} failed ({rc}): {lib().mmt_last_error().decode(errors='replace')}")
        return rc
    if rc != 0:
        msg = lib().mmt_last_error().decode(errors="replace")
        raise MMTError(f"{name} failed ({rc}): {msg}")
    return rc


def exported_symbols() -> list[str]:
    return ["mmt_last_error", *SIGNATURES.keys()]


WS_TOME_MATCH = 1  # mmt_workspace_size op codes (include/mmt_api.h)


def workspace_size(op: int, *dims: int) -> int:
    arr = (ctypes.c_int64 * len(dims))(*dims)
    return call("mmt_workspace_size", op, arr, len(dims))


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_ptr() -> int:
    import torch
    return torch.cuda.current_stream().cuda_stream
