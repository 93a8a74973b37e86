"""Parameter-tree and checkpoint interchange.

* ``to_flax_params(model)`` / ``load_flax_params(model, tree)``: this build's flat ParamStore <->
  the nested ``params`` tree the reference's Flax ``Octo`` module produces (octo.py:58-84 setup
  attributes, ``nn.compact`` auto-names), with the reference's layouts: Dense kernels (in, out);
  the transformer blocks scan-stacked on axis 0 under ``ScanEncoder1DBlock_0``
  (attention.py:103-109, ``variable_axes={'params': 0}``); ``SelfAttention`` query/key/value
  kernels (D, H, Dh) and out (H, Dh, D) (flax.linen.MultiHeadDotProductAttention); convolution
  kernels (kh, kw, cin, cout); position embeddings with their leading 1 axis.
* ``flax_msgpack_dumps`` / ``flax_msgpack_loads``: the ``flax.serialization.to_bytes`` wire format
  (msgpack maps, ndarrays as ext type 1 = packed (shape, dtype name, raw bytes), numpy scalars as
  ext type 3, chunked big arrays), so a tree saved by ``flax.serialization.to_bytes(params)`` loads
  here and the reverse. Nothing is unpickled.
* ``hf_t5_to_store(t5, state_dict)``: weights of a transformers ``T5EncoderModel`` (torch state
  dict, e.g. a local t5-base) into the frozen T5 store (the reference's text encoder is
  ``FlaxT5EncoderModel(AutoConfig.from_pretrained('t5-base'))``, t5_base.py:11).
* ``save_train_state`` / ``load_train_state``: resume files (flat fp32 master, AdamW moments, RNG
  state) via ``torch.save`` of plain tensors, loaded with ``weights_only=True``.

Parity: no checkpoint of the reference exists anywhere (its orbax dependency is unused,
pyproject.toml:33-34), so the tree layout is restated from the Flax module definitions and is
"parity unpinned" at the name level; where the name of a ``setup``-assigned submodule with an
explicit ``name=`` (the image tokenizer's position embeddings) is ambiguous, loading accepts both
candidates. The stem's 3x3 SAME convolutions act on a 1x1 map here, so only their centre tap is
stored; export writes the full (3, 3, C, C) kernel with zero outer taps and import reads the
centre tap (exact for this geometry).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Tuple

import msgpack
import numpy as np
import torch

# ---------------------------------------------------------------- flax msgpack wire format
_EXT_NDARRAY, _EXT_COMPLEX, _EXT_NPSCALAR = 1, 2, 3
_CHUNK_KEY = "__msgpack_chunked_array__"
MAX_CHUNK = 2 ** 30


def _ndarray_to_bytes(a: np.ndarray) -> bytes:
    a = np.ascontiguousarray(a)
    return msgpack.packb((a.shape, a.dtype.name, a.tobytes()), use_bin_type=True)


def _ndarray_from_bytes(b: bytes) -> np.ndarray:
    shape, dtype_name, buf = msgpack.unpackb(b, raw=True)
    name = dtype_name.decode() if isinstance(dtype_name, bytes) else dtype_name
    return np.frombuffer(buf, dtype=np.dtype(name)).reshape(shape).copy()


def _default(obj):
    if isinstance(obj, np.ndarray):
        return msgpack.ExtType(_EXT_NDARRAY, _ndarray_to_bytes(obj))
    if isinstance(obj, np.generic):
        return msgpack.ExtType(_EXT_NPSCALAR, msgpack.packb((obj.dtype.name, obj.tobytes()),
                                                            use_bin_type=True))
    if isinstance(obj, torch.Tensor):
        return _default(obj.detach().cpu().numpy())
    raise TypeError(f"cannot serialise {type(obj)}")


def _ext_hook(code, data):
    if code == _EXT_NDARRAY:
        return _ndarray_from_bytes(data)
    if code == _EXT_COMPLEX:
        re, im = msgpack.unpackb(data)
        return complex(re, im)
    if code == _EXT_NPSCALAR:
        name, buf = msgpack.unpackb(data, raw=True)
        return np.frombuffer(buf, dtype=np.dtype(name.decode() if isinstance(name, bytes) else name))[0]
    return msgpack.ExtType(code, data)


def _chunk(tree):
    """Large arrays as {__msgpack_chunked_array__, shape, chunks} (flax _chunk_array_leaves)."""
    if isinstance(tree, dict):
        return {k: _chunk(v) for k, v in tree.items()}
    if isinstance(tree, np.ndarray) and tree.nbytes > MAX_CHUNK:
        flat = tree.reshape(-1)
        n = max(1, MAX_CHUNK // max(flat.itemsize, 1))
        chunks = {str(i): flat[j:j + n] for i, j in enumerate(range(0, flat.size, n))}
        # flax stores the shape as a {"0": d0, "1": d1, ...} map (strict_types packing)
        return {_CHUNK_KEY: True, "shape": {str(i): int(d) for i, d in enumerate(tree.shape)},
                "chunks": chunks}
    return tree


def _unchunk(tree):
    if isinstance(tree, dict):
        if tree.get(_CHUNK_KEY):
            chunks = tree["chunks"]
            parts = [chunks[str(i)] for i in range(len(chunks))]
            shape = tree["shape"]
            if isinstance(shape, dict):
                shape = tuple(shape[str(i)] for i in range(len(shape)))
            return np.concatenate(parts).reshape(shape)
        return {k: _unchunk(v) for k, v in tree.items()}
    return tree


def flax_msgpack_dumps(tree: dict) -> bytes:
    return msgpack.packb(_chunk(tree), default=_default, strict_types=True, use_bin_type=True)


def flax_msgpack_loads(data: bytes) -> dict:
    return _unchunk(msgpack.unpackb(data, ext_hook=_ext_hook, raw=False, strict_map_key=False))


# ---------------------------------------------------------------- tree helpers
def _get(tree: dict, path: str):
    node = tree
    for k in path.split("/"):
        if not isinstance(node, dict) or k not in node:
            return None
        node = node[k]
    return node


def _set(tree: dict, path: str, value):
    keys = path.split("/")
    node = tree
    for k in keys[:-1]:
        node = node.setdefault(k, {})
    node[keys[-1]] = value


def flatten_tree(tree: dict, prefix: str = "") -> Dict[str, np.ndarray]:
    out = {}
    for k, v in tree.items():
        p = f"{prefix}/{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(flatten_tree(v, p))
        else:
            out[p] = v
    return out


# ---------------------------------------------------------------- layout rules
# A rule maps one of this build's parameters to one Flax leaf: (flax path candidates, export
# transform ours -> flax, import transform flax -> ours). Scan-stacked block leaves are handled
# separately (one Flax leaf = all blocks).
Rule = Tuple[List[str], Callable[[np.ndarray], np.ndarray], Callable[[np.ndarray], np.ndarray]]


def _dense_T(a):
    return np.ascontiguousarray(a.T)


def _ident(a):
    return np.ascontiguousarray(a)


def _lead1(a):
    return np.ascontiguousarray(a[None])


def _drop1(a):
    return np.ascontiguousarray(a[0])


def _rules(model) -> Dict[str, Rule]:
    rules: Dict[str, Rule] = {}
    it = model.image_tokenizer
    rn = it.resnet
    C_img = it.image_size[2]
    E = "image_encoder"
    for which in ("row", "col"):
        rules[f"ImageTokenizer_0/image_{which}_position_embedding/embedding"] = (
            [f"{E}/{which}_embeddings/embedding", f"{E}/image_{which}_position_embedding/embedding"],
            _ident, _ident)
    ef = f"{E}/embedding_function"
    kh, kw, C = rn.kh, rn.kw, rn.C
    rules["ImageTokenizer_0/ResNetV2Block_0/Conv_0/kernel"] = (
        [f"{ef}/Conv_0/kernel"],
        lambda a: np.ascontiguousarray(a.T.reshape(kh, kw, C_img, C)),
        lambda a: np.ascontiguousarray(a.reshape(kh * kw * C_img, C).T))
    rules["ImageTokenizer_0/ResNetV2Block_0/Conv_0/bias"] = ([f"{ef}/Conv_0/bias"], _ident, _ident)
    for i in range(rn.num_blocks):
        for leaf in ("scale", "bias"):
            rules[f"ImageTokenizer_0/ResNetV2Block_0/GroupNorm_{i}/{leaf}"] = (
                [f"{ef}/GroupNorm_{i}/{leaf}"], _ident, _ident)

        def exp3(a):
            k = np.zeros((3, 3, a.shape[1], a.shape[0]), a.dtype)
            k[1, 1] = a.T
            return k
        rules[f"ImageTokenizer_0/ResNetV2Block_0/Conv_{i + 1}/kernel"] = (
            [f"{ef}/Conv_{i + 1}/kernel"], exp3, lambda a: np.ascontiguousarray(a[1, 1].T))
        rules[f"ImageTokenizer_0/ResNetV2Block_0/Conv_{i + 1}/bias"] = (
            [f"{ef}/Conv_{i + 1}/bias"], _ident, _ident)
    rules["ImageTokenizer_0/ResNetV2Block_0/Dense_0/kernel"] = ([f"{ef}/Dense_0/kernel"], _dense_T, _dense_T)
    rules["ImageTokenizer_0/ResNetV2Block_0/Dense_0/bias"] = ([f"{ef}/Dense_0/bias"], _ident, _ident)
    rules["AddPositionEmbedding_0/pos_embedding"] = (["readout_encoder/pos_embedding"], _lead1, _drop1)
    rules["StackedEncoder1DBlock_0/posembed_input/pos_embedding"] = (
        ["attention_blocks/posembed_input/pos_embedding"], _lead1, _drop1)
    if model.text_proj is not None:  # this build's projection of T5 features to D (no reference twin)
        rules["TextProjection_0/kernel"] = (["TextProjection_0/kernel"], _dense_T, _dense_T)
        rules["TextProjection_0/bias"] = (["TextProjection_0/bias"], _ident, _ident)
    hd = "diffusion_action_head/denoiser"
    ours = "diffusion_action_head/OctoDenoise_0"
    rules[f"{ours}/FourierFeatures_0/fourier_kernel"] = ([f"{hd}/FourierFeatures_0/fourier_kernel"],
                                                         _ident, _ident)
    for blk in ("FourierFeatures_0/MLPBlock_0", "MLPBlock_0"):
        for d in ("Dense_0", "Dense_1"):
            rules[f"{ours}/{blk}/{d}/kernel"] = ([f"{hd}/{blk}/{d}/kernel"], _dense_T, _dense_T)
            rules[f"{ours}/{blk}/{d}/bias"] = ([f"{hd}/{blk}/{d}/bias"], _ident, _ident)
    return rules


SCAN = "attention_blocks/ScanEncoder1DBlock_0"


def _block_leaves(model):
    """(flax leaf under SCAN, per-block export fn(block) -> array, import fn(block, array))."""
    D, H = model.D, model.cfg.num_heads
    Dh = D // H
    out = []
    for ln in ("LayerNorm_0", "LayerNorm_1"):
        for leaf in ("scale", "bias"):
            attr = "ln0" if ln == "LayerNorm_0" else "ln1"
            out.append((f"{ln}/{leaf}",
                        (lambda b, attr=attr, leaf=leaf: getattr(getattr(b, attr), leaf).data),
                        None))
    for j, n in enumerate(("query", "key", "value")):
        out.append((f"SelfAttention_0/{n}/kernel",
                    (lambda b, j=j: b.qkv.w.data[j * D:(j + 1) * D].T.reshape(D, H, Dh)),
                    (lambda b, a, j=j: b.qkv.w.data[j * D:(j + 1) * D].copy_(
                        torch.from_numpy(a.reshape(D, H * Dh).T.copy())))))
        out.append((f"SelfAttention_0/{n}/bias",
                    (lambda b, j=j: b.qkv.b.data[j * D:(j + 1) * D].reshape(H, Dh)),
                    (lambda b, a, j=j: b.qkv.b.data[j * D:(j + 1) * D].copy_(
                        torch.from_numpy(a.reshape(-1).copy())))))
    out.append(("SelfAttention_0/out/kernel", lambda b: b.out.w.data.T.reshape(H, Dh, D),
                lambda b, a: b.out.w.data.copy_(torch.from_numpy(a.reshape(H * Dh, D).T.copy()))))
    out.append(("SelfAttention_0/out/bias", lambda b: b.out.b.data, None))
    for d, attr in (("Dense_0", "dense"), ("Dense_1", "dense_out")):
        out.append((f"MLPBlock_0/{d}/kernel", lambda b, attr=attr: getattr(b.mlp, attr).w.data.T,
                    lambda b, a, attr=attr: getattr(b.mlp, attr).w.data.copy_(
                        torch.from_numpy(a.T.copy()))))
        out.append((f"MLPBlock_0/{d}/bias", lambda b, attr=attr: getattr(b.mlp, attr).b.data, None))
    return out


def _generic_import(leaf: str):
    """Import of a block leaf whose layout equals ours (LayerNorm, biases)."""
    def imp(b, a):
        if leaf.startswith("LayerNorm"):
            ln = b.ln0 if leaf.startswith("LayerNorm_0") else b.ln1
            t = ln.scale if leaf.endswith("scale") else ln.bias
        elif leaf == "SelfAttention_0/out/bias":
            t = b.out.b
        else:
            t = (b.mlp.dense if "Dense_0" in leaf else b.mlp.dense_out).b
        t.data.copy_(torch.from_numpy(np.ascontiguousarray(a).reshape(t.data.shape)))
    return imp


def to_flax_params(model) -> dict:
    """Nested {'name': ... ndarray} tree in the reference's Flax layout (fp32)."""
    tree: dict = {}
    by_name = model.store.by_name
    for name, (paths, exp, _imp) in _rules(model).items():
        _set(tree, paths[0], exp(by_name[name].data.detach().float().cpu().numpy()))
    blocks = model.stack.blocks
    for leaf, exp, _imp in _block_leaves(model):
        arr = np.stack([exp(b).detach().float().cpu().numpy() for b in blocks])
        _set(tree, f"{SCAN}/{leaf}", np.ascontiguousarray(arr.astype(np.float32)))
    return tree


def load_flax_params(model, tree: dict, strict: bool = True) -> List[str]:
    """Load a reference-layout tree (e.g. flax_msgpack_loads of flax.serialization.to_bytes) into
    the model's master weights and refresh the bf16 shadow. Returns the names not found (raises
    if strict and any is missing or mis-shaped)."""
    missing = []
    by_name = model.store.by_name
    with torch.no_grad():
        for name, (paths, _exp, imp) in _rules(model).items():
            leaf = next((v for v in (_get(tree, p) for p in paths) if v is not None), None)
            if leaf is None:
                missing.append(name)
                continue
            p = by_name[name]
            val = imp(np.asarray(leaf, dtype=np.float32))
            if tuple(val.shape) != tuple(p.shape):
                raise ValueError(f"{name}: tree leaf {paths[0]} gives {val.shape}, expected {p.shape}")
            p.data.copy_(torch.from_numpy(val).to(p.data.device))
        blocks = model.stack.blocks
        for leaf, _exp, imp in _block_leaves(model):
            arr = _get(tree, f"{SCAN}/{leaf}")
            if arr is None:
                missing.append(f"{SCAN}/{leaf}")
                continue
            arr = np.asarray(arr, dtype=np.float32)
            if arr.shape[0] != len(blocks):
                raise ValueError(f"{leaf}: {arr.shape[0]} stacked blocks, model has {len(blocks)}")
            fn = imp or _generic_import(leaf)
            for i, b in enumerate(blocks):
                cpu = _CpuBlock(b)
                fn(cpu, arr[i])
                cpu.flush()
    if strict and missing:
        raise KeyError(f"parameters missing from the tree: {missing[:8]}")
    model.store.sync_shadow()
    return missing


class _CpuBlock:
    """Host staging view of one Encoder1DBlock's parameters (import functions write into CPU
    copies; flush() uploads them)."""

    def __init__(self, blk):
        self._blk = blk
        self._copies = []

        def stage(layer_obj, attrs):
            class _NS:
                pass
            ns = _NS()
            for a in attrs:
                p = getattr(layer_obj, a)
                if p is None:
                    setattr(ns, a, None)
                    continue
                host = _HostParam(p)
                self._copies.append(host)
                setattr(ns, a, host)
            return ns
        self.ln0 = stage(blk.ln0, ("scale", "bias"))
        self.ln1 = stage(blk.ln1, ("scale", "bias"))
        self.qkv = stage(blk.qkv, ("w", "b"))
        self.out = stage(blk.out, ("w", "b"))

        class _M:
            pass
        self.mlp = _M()
        self.mlp.dense = stage(blk.mlp.dense, ("w", "b"))
        self.mlp.dense_out = stage(blk.mlp.dense_out, ("w", "b"))

    def flush(self):
        for h in self._copies:
            h.flush()


class _HostParam:
    def __init__(self, p):
        self._p = p
        self.data = p.data.detach().float().cpu().clone()

    def flush(self):
        self._p.data.copy_(self.data.to(self._p.data.device))


# ---------------------------------------------------------------- T5 (frozen text encoder)
def hf_t5_to_store(t5, state_dict: Dict[str, torch.Tensor]) -> None:
    """transformers T5EncoderModel state dict (torch names) -> the frozen bf16 T5 store."""
    pre = t5.store.params[0].name.split("/")[0]
    by = t5.store.by_name
    put = {f"{pre}/shared/embedding": state_dict["shared.weight"],
           f"{pre}/relative_attention_bias":
               state_dict["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"],
           f"{pre}/final_layer_norm": state_dict["encoder.final_layer_norm.weight"]}
    i = 0
    while f"encoder.block.{i}.layer.0.layer_norm.weight" in state_dict:
        b, p = f"encoder.block.{i}.layer", f"{pre}/block/{i}"
        put[f"{p}/layer_0/layer_norm"] = state_dict[f"{b}.0.layer_norm.weight"]
        put[f"{p}/SelfAttention/qkv"] = torch.cat(
            [state_dict[f"{b}.0.SelfAttention.{n}.weight"] for n in "qkv"], 0)
        put[f"{p}/SelfAttention/o"] = state_dict[f"{b}.0.SelfAttention.o.weight"]
        put[f"{p}/layer_1/layer_norm"] = state_dict[f"{b}.1.layer_norm.weight"]
        put[f"{p}/DenseReluDense/wi"] = state_dict[f"{b}.1.DenseReluDense.wi.weight"]
        put[f"{p}/DenseReluDense/wo"] = state_dict[f"{b}.1.DenseReluDense.wo.weight"]
        i += 1
    for name, val in put.items():
        p = by[name]
        if tuple(val.shape) != tuple(p.shape):
            raise ValueError(f"{name}: {tuple(val.shape)} != {p.shape}")
        p.bf16.copy_(val.to(p.bf16.device, torch.bfloat16))


# ---------------------------------------------------------------- resume files
def save_train_state(path: str, train_state) -> None:
    s = train_state.model.store
    torch.save({"flat": s.flat.cpu(), "m": s.m.cpu(), "v": s.v.cpu(),
                "rng": train_state.rng.cpu(), "sample_offset": torch.tensor(train_state.sample_offset),
                "names": [p.name for p in s.params], "n": torch.tensor(s.n)}, path)


def load_train_state(path: str, train_state) -> None:
    d = torch.load(path, map_location="cpu", weights_only=True)
    s = train_state.model.store
    if d["names"] != [p.name for p in s.params] or int(d["n"]) != s.n:
        raise ValueError("checkpoint parameter layout differs from the model's")
    s.flat.copy_(d["flat"].to(s.flat.device))
    s.m.copy_(d["m"].to(s.m.device))
    s.v.copy_(d["v"].to(s.v.device))
    train_state.rng.copy_(d["rng"].to(train_state.rng.device))
    train_state.sample_offset = int(d["sample_offset"])
    s.sync_shadow()
