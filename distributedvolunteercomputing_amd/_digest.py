"""Source digests of the two in-tree extensions (no torch import).

``_build`` links the digest of the sources it compiled into each shared object
(``_C.source_digest()``, ``_native.source_digest()``); the loaders (``ops/_lib.py``,
``_native_loader.py``) recompute it from the sources next to them and refuse an extension built
from other sources. The ``.so`` files are git-ignored and travel prebuilt in the repo snapshot, so
without this an extension left over from an older tree would load silently.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"


def source_files(kind: str) -> list[Path]:
    if kind == "C":
        k = CSRC / "kernels"
        return sorted(list(k.glob("*.hip")) + list(k.glob("*.h")) + list(CSRC.glob("bindings*.cpp")))
    if kind == "native":
        rt = CSRC / "runtime"
        return sorted(list(rt.glob("*.cpp")) + list(rt.glob("*.h")))
    raise ValueError(kind)


def source_digest(kind: str) -> str | None:
    """sha256 (16 hex) over the names and bytes of the extension's sources; None when the sources
    are not shipped next to the package (nothing to compare against)."""
    files = source_files(kind)
    if not files:
        return None
    h = hashlib.sha256(kind.encode())
    for p in files:
        h.update(p.name.encode())
        h.update(b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


class StaleExtension(RuntimeError):
    pass


def check(mod, kind: str) -> None:
    """Raise StaleExtension when `mod` was built from sources other than the ones in the tree."""
    want = source_digest(kind)
    if want is None:
        return
    got = getattr(mod, "source_digest", None)
    got = got() if callable(got) else None
    if got != want:
        raise StaleExtension(
            f"distributedvolunteercomputing_amd.{'_C' if kind == 'C' else '_native'} was built from other "
            f"sources (extension digest {got!r}, tree {want!r}): rebuild with "
            f"`python -m distributedvolunteercomputing_amd._build`")
