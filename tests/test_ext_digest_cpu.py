"""A prebuilt extension built from other sources is refused.

The ``.so`` files are git-ignored and travel prebuilt with the repo snapshot; ``_build`` links the
digest of the sources it compiled into each, and the loaders compare it with the tree's sources.
"""
import types

import pytest

from distributedvolunteercomputing_amd import _digest


def _fake(d):
    return types.SimpleNamespace(source_digest=lambda: d)


@pytest.mark.parametrize("kind", ["C", "native"])
def test_stale_digest_is_refused(kind):
    want = _digest.source_digest(kind)
    assert want and len(want) == 16
    _digest.check(_fake(want), kind)  # the matching build loads
    with pytest.raises(_digest.StaleExtension, match="rebuild"):
        _digest.check(_fake("0" * 16), kind)
    with pytest.raises(_digest.StaleExtension):
        _digest.check(types.SimpleNamespace(), kind)  # built before digests existed


def test_digest_follows_every_source(tmp_path, monkeypatch):
    base = _digest.source_digest("C")
    src = tmp_path / "csrc"
    (src / "kernels").mkdir(parents=True)
    for p in _digest.source_files("C"):
        dst = (src / "kernels" / p.name) if p.parent.name == "kernels" else (src / p.name)
        dst.write_bytes(p.read_bytes())
    monkeypatch.setattr(_digest, "CSRC", src)
    assert _digest.source_digest("C") == base
    k = sorted((src / "kernels").glob("*.hip"))[0]
    k.write_bytes(k.read_bytes() + b"\n// edited\n")
    assert _digest.source_digest("C") != base


def test_built_extensions_match_the_tree():
    from distributedvolunteercomputing_amd import _native_loader
    from distributedvolunteercomputing_amd.ops import _lib

    if not _lib.available():
        pytest.skip(f"_C not built here: {_lib._ERR!r}")
    assert _lib.native().source_digest() == _digest.source_digest("C")
    assert _native_loader.native().source_digest() == _digest.source_digest("native")
