"""Which GPU a volunteer process uses.

The reference runs its detector on the CPU of whatever machine the volunteer is on
(/root/reference/worker.py:194). Here each volunteer wants a GPU of its own: under a launcher
(torchrun) that is LOCAL_RANK's GPU; volunteers started by hand on one node (``python worker.py``
N times) claim the first GPU that no other volunteer on this host holds, through an advisory file
lock per GPU that lives as long as the process (the kernel drops it when the process exits, also
on a crash, so a dead volunteer never keeps its GPU claimed). With more volunteers than GPUs the
extra ones share, spread by process id.
"""
from __future__ import annotations

import fcntl
import os
import tempfile

_HELD: list = []  # open lock files: the claim lasts as long as this process


def claim_device(lock_dir: str | None = None) -> str:
    """'cuda:N' for this volunteer (or 'cpu' without GPUs); does not initialise the GPU."""
    import torch

    n = torch.cuda.device_count()  # does not create a HIP context on this image
    if n == 0:
        return "cpu"
    if os.environ.get("LOCAL_RANK") is not None:
        return f"cuda:{int(os.environ['LOCAL_RANK']) % n}"
    d = lock_dir or os.path.join(tempfile.gettempdir(), f"vcx-gpu-claims-{os.getuid()}")
    os.makedirs(d, exist_ok=True)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES") or ""
    tag = vis.replace(",", "_") or "all"  # claims are per visible-device set
    for i in range(n):
        f = open(os.path.join(d, f"{tag}-{i}.lock"), "a")
        try:
            fcntl.flock(f.fileno(), fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            f.close()
            continue
        _HELD.append(f)
        return f"cuda:{i}"
    return f"cuda:{os.getpid() % n}"


def release_all():
    """Drop this process's claims (tests)."""
    while _HELD:
        f = _HELD.pop()
        try:
            fcntl.flock(f.fileno(), fcntl.LOCK_UN)
        finally:
            f.close()
