"""Multi-process helpers for CPU (gloo) distributed tests."""
from __future__ import annotations

import datetime
import multiprocessing as mp
import os
import socket
import traceback


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_store(rank: int, world: int, port: int, wait_workers: bool = False, timeout_s: float = 60):
    import torch.distributed as dist

    return dist.TCPStore("127.0.0.1", port, world if wait_workers else None, rank == 0,
                         timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=wait_workers)


def _entry(fn, rank, world, port, q, args):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    try:
        import torch

        torch.set_num_threads(1)
        res = fn(rank, world, port, *args)
        q.put((rank, "ok", res))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, "err", f"{e!r}\n{traceback.format_exc()}"))


def run(fn, world: int, *args, timeout: float = 120.0, expect_exit=()):
    """Run fn(rank, world, port, *args) in `world` spawned processes; return {rank: result}.
    Ranks listed in expect_exit may die without reporting."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args), daemon=True) for r in range(world)]
    for p in procs:
        p.start()
    out, errs = {}, []
    need = set(range(world)) - set(expect_exit)
    import queue as _q
    import time

    t0 = time.time()
    while not need.issubset(set(out) | {r for r, _ in errs}) and time.time() - t0 < timeout:
        try:
            r, st, res = q.get(timeout=1.0)
        except _q.Empty:
            continue
        if st == "ok":
            out[r] = res
        else:
            errs.append((r, res))
    for p in procs:
        p.join(timeout=5)
        if p.is_alive():
            p.kill()
    if errs:
        raise AssertionError("worker failures:\n" + "\n".join(f"[rank {r}] {e}" for r, e in errs))
    if not need.issubset(out):
        raise AssertionError(f"timeout: only ranks {sorted(out)} finished")
    return out
