"""Probe: can two ranks share one GPU with RCCL (ProcessGroupNCCL) on this box? Used to decide
whether the RCCL-only PeerGroup paths (per-generation communicators, abort) can be exercised on a
one-GPU machine. Prints the outcome; exits 0 either way unless the child hangs (killed by timeout)."""
import datetime
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(rank, port, q):
    try:
        torch.cuda.set_device(0)
        store = dist.TCPStore("127.0.0.1", port, 2, rank == 0, timeout=datetime.timedelta(seconds=30))
        opts = dist.ProcessGroupNCCL.Options()
        opts._timeout = datetime.timedelta(seconds=20)
        pg = dist.ProcessGroupNCCL(store, rank, 2, opts)
        t = torch.full((4,), float(rank + 1), device="cuda:0")
        pg.allreduce([t]).wait()
        torch.cuda.synchronize()
        q.put((rank, "ok", t.tolist()))
    except Exception as e:  # noqa: BLE001
        q.put((rank, "err", repr(e)[:300]))


if __name__ == "__main__":
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=child, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = []
    for _ in range(2):
        try:
            res.append(q.get(timeout=60))
        except Exception:  # noqa: BLE001
            res.append(("?", "timeout", None))
    for p in ps:
        p.join(5)
        if p.is_alive():
            p.kill()
    print("RCCL two ranks on one GPU:", res, flush=True)
