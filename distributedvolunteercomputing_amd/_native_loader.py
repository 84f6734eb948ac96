"""Loads the C++ host runtime ``_native`` (transport, scheduler, reorder index)."""
from __future__ import annotations

import importlib

_mod = None


def native():
    global _mod
    if _mod is None:
        try:
            _mod = importlib.import_module("distributedvolunteercomputing_amd._native")
        except ImportError as e:
            raise RuntimeError(
                "distributedvolunteercomputing_amd._native (C++ runtime) is not built: "
                "run `python -m distributedvolunteercomputing_amd._build --only native`"
            ) from e
    return _mod
