"""Reference-signature module plumbing shared by the class-level API.

The reference's modules are Flax dataclasses whose fields are Hydra config nodes
(``DictConfig``), instantiated inside ``__call__`` (``attention.py:20-119``,
``image_tokenizer.py:140-309``, ``diffusion.py:30-143``), and whose parameters are created on the
first call from the input shapes (``nn.compact``). The build's modules keep those constructors
and call signatures; a field may arrive as

* a raw YAML node (a dict with ``_target_``; ``instantiate(..., _recursive_=False)`` as
  ``octo.py:76-84`` does),
* a :class:`~.config_loader.LayerSpec` (``instantiate`` of a ``flax.linen.*`` / initializer node),
* an already-built build module (``instantiate`` with ``_recursive_=True``), or a plain value.

:func:`spec` normalises the first two to a LayerSpec. Parameters live in a flat
:class:`~.params.ParamStore`: a module either binds into a caller's store (``bind``: the Octo
model declares every component in one store, so one AdamW launch and one all-reduce cover
everything) or, on its first call with nothing bound, creates, initialises (seeded, the Flax
initialisers) and uploads its own, as ``Module.init`` would.
"""
from __future__ import annotations

import math
from typing import Any, Optional

import torch

from .config_loader import LayerSpec, instantiate
from .params import ParamStore, const, he_normal, normal, variance_scaling_normal


def spec(node) -> Any:
    """A config field as the build consumes it: dict nodes with a ``_target_`` instantiated
    (LayerSpec for Flax layers / initializers, build modules for build targets), the rest as is."""
    if isinstance(node, dict) and "_target_" in node:
        return instantiate(node, _recursive_=False)
    return node


def sget(node, key: str, default=None):
    """Field ``key`` of a LayerSpec / dict / module attribute (``default`` when absent)."""
    node = spec(node)
    if node is None:
        return default
    if isinstance(node, LayerSpec):
        v = node.kwargs.get(key, default)
    elif isinstance(node, dict):
        v = node.get(key, default)
    else:
        v = getattr(node, key, default)
    return default if v is None else v


def merge_param(name: str, a, b):
    """flax.linen.module.merge_param: a value set in the constructor OR passed to the call, never
    both, never neither (the reference's Encoder1DBlock train / mask, attention.py:54-55)."""
    a_set, b_set = a is not None, b is not None
    if a_set and b_set:
        raise ValueError(f'If "{name}" is passed to the constructor, it must not be passed to the call')
    if not a_set and not b_set:
        raise ValueError(f'"{name}" must be set either in the constructor or in the call')
    return a if a_set else b


def init_from_spec(init, flax_shape, default=None):
    """A Flax initializer node / LayerSpec / callable as a ParamStore initialiser for a parameter
    of Flax shape ``flax_shape`` (kernels (..., in, out)). Known targets: he_normal, normal,
    variance_scaling (normal, fan_in), zeros, ones, lecun_normal, glorot/xavier_normal. A plain
    callable is taken as a ParamStore initialiser ``init(tensor, generator)`` (params.py)."""
    init = spec(init)
    if init is None:
        return default if default is not None else he_normal(flax_shape)
    if callable(init) and not isinstance(init, LayerSpec):
        return init
    name = init.target.rsplit(".", 1)[-1]
    kw = init.kwargs
    if name == "he_normal":
        return he_normal(flax_shape)
    if name == "normal":
        return normal(float(kw.get("stddev", 0.01) or 0.01))
    if name == "zeros":
        return const(0.0)
    if name == "ones":
        return const(1.0)
    if name == "variance_scaling":
        if kw.get("distribution", "normal") != "normal" or kw.get("mode", "fan_in") != "fan_in":
            raise NotImplementedError(f"variance_scaling {kw} (the build implements normal / fan_in)")
        return variance_scaling_normal(float(kw.get("scale", 1.0)), flax_shape)
    if name in ("lecun_normal",):
        return variance_scaling_normal(1.0, flax_shape)
    if name in ("glorot_normal", "xavier_normal"):
        fan_in = flax_shape[-2] if len(flax_shape) > 1 else flax_shape[0]
        fan_out = flax_shape[-1]
        return normal(math.sqrt(2.0 / (fan_in + fan_out)))
    raise NotImplementedError(f"initializer {init.target!r}")


class Bindable:
    """Lazy parameter binding: ``bind(store, name, ...)`` declares the parameters in a caller's
    store; ``_ensure(device, ...)`` (first call) creates a private store when nothing is bound."""
    _store: Optional[ParamStore] = None
    _name: str = ""

    @property
    def bound(self) -> bool:
        return self._store is not None

    @property
    def store(self) -> Optional[ParamStore]:
        return self._store

    def _declare(self, store: ParamStore, name: str, *dims):  # pragma: no cover - interface
        raise NotImplementedError

    def bind(self, store: ParamStore, name: str, *dims):
        if self._store is not None:
            raise RuntimeError(f"{type(self).__name__} is already bound to a parameter store")
        self._declare(store, name, *dims)
        self._store, self._name = store, name
        return self

    def _ensure(self, device, *dims, seed: int = 0):
        if self._store is None:
            st = ParamStore()
            self.bind(st, type(self).__name__ + "_0", *dims)
            st.materialize(torch.device(device), seed)
        return self

    @property
    def params(self):
        """The module's parameters by name (views of the store's fp32 master)."""
        if self._store is None:
            return {}
        pre = self._name + "/"
        return {p.name: p.data for p in self._store.params if p.name.startswith(pre)}
