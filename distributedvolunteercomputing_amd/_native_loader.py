"""Loads the C++ host runtime ``_native`` (transport, scheduler, reorder index)."""
from __future__ import annotations

import importlib

from . import _digest

_mod = None


def native():
    global _mod
    if _mod is None:
        try:
            mod = importlib.import_module("distributedvolunteercomputing_amd._native")
        except ImportError as e:
            raise RuntimeError(
                "distributedvolunteercomputing_amd._native (C++ runtime) is not built: "
                "run `python -m distributedvolunteercomputing_amd._build --only native`"
            ) from e
        _digest.check(mod, "native")  # refuse a runtime built from other sources
        _mod = mod
    return _mod
