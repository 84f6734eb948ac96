"""Loader for the in-tree gfx950 extension ``_C``.

Policy: GPU tensors ALWAYS go through the HIP kernels. If the extension is missing or fails
to load, GPU ops raise immediately (no silent eager fallback on a GPU box). CPU tensors use
the plain-PyTorch reference implementations in each op module; those references double as
the numerics oracle in the tests.
"""
from __future__ import annotations

import importlib

from .. import _digest, config

_C = None
_ERR: Exception | None = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        mod = importlib.import_module("distributedvolunteercomputing_amd._C")
        _digest.check(mod, "C")  # refuse an extension built from other sources (stale prebuilt .so)
        _C = mod
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e


def native():
    """Return the compiled module or raise a loud error explaining how to build it."""
    _load()
    if _C is None:
        raise RuntimeError(
            "distributedvolunteercomputing_amd._C (gfx950 HIP kernels) is not built or failed to load: "
            f"{_ERR!r}. Build it with `python -m distributedvolunteercomputing_amd._build`."
        )
    return _C


def available() -> bool:
    _load()
    return _C is not None




def use_native(t) -> bool:
    """True when tensor `t` lives on the GPU (then the native kernel is mandatory)."""
    if config.get().force_reference_ops:
        return False
    return bool(getattr(t, "is_cuda", False))


def grad_buffer(p):
    """p.grad when it is a preset contiguous gradient buffer of p's shape/dtype (the flat-buffer
    view installed by parallel/flat_params.py): backward kernels then ADD their result straight
    into it and hand autograd ``None`` for that input, which skips autograd's accumulation pass."""
    g = getattr(p, "grad", None) if p is not None else None
    if g is not None and g.dtype == p.dtype and g.is_contiguous() and g.shape == p.shape and g.is_cuda:
        return g
    return None


class reference_ops:
    """Context manager: run the plain-PyTorch reference path even for GPU tensors.
    Used ONLY by the numerics tests to build an oracle on the same device."""

    def __enter__(self):
        self._old = config.get().force_reference_ops
        config.update(force_reference_ops=True)

    def __exit__(self, *exc):
        config.update(force_reference_ops=self._old)
