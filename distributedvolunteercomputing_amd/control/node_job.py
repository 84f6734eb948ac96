"""One-node video job: every GPU of the node is a volunteer, chunks move GPU-to-GPU.

Launched one process per GPU (``torchrun --nproc-per-node N``, or any launcher that sets
RANK / WORLD_SIZE / LOCAL_RANK). Rank 0 hosts the coordinator with ``data_plane="p2p"`` and is
the requester; every other rank joins it as a worker volunteer. It is the ordinary volunteer
API (join / request / stop / end verbs, leases, re-dispatch of a dead worker's chunks) on the
peer-to-peer plane — not a separate static job: a worker that dies mid-job has its chunks
re-dispatched to the others, a volunteer from another machine can join the same coordinator.

Reference analog: starting server.py on one machine and worker.py on every other
(/root/reference/server.py:159-172, worker.py:283-307), with the chunk bytes taken off the
coordinator's host path.
"""
from __future__ import annotations

import datetime
import os
import time

import torch
import torch.distributed as dist

from .. import config
from .coordinator import coordinator
from .peer import client

DONE_KEY = "vcx/node_job/done"


def shared_root_of(source: str) -> str | None:
    """The directory of a memory-mapped .npy source (``<file>.npy`` or ``<file>.npy@<total>``), else None."""
    f = source.rsplit("@", 1)[0] if "@" in source else source
    return os.path.dirname(os.path.realpath(f)) if f.endswith(".npy") and os.path.isfile(f) else None


def run_node_job(source: str, out_dir: str, *, engine_factory, chunk: int = 100, control_port: int = 9999,
                 store_port: int = 29612, lease_s: float = 10.0, out_ext: str = ".y4m", preresize: bool = True,
                 timeout_s: float = 3600.0, shared_source: bool = True):
    """Run this rank's part; rank 0 returns the job stats, workers the number of frames served.

    shared_source: with an .npy source every volunteer of the node reads its chunks' frames from the file
    itself (index windows on the p2p plane, peer._Window): the raw frames cross each worker GPU's own host
    link instead of all of them crossing the requester's."""
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    root = shared_root_of(source) if shared_source else None
    if root is not None and not config.get().shared_source_root:
        config.update(shared_source_root=root)
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    # job-control store (this job's "done" flag only; pair groups rendezvous on the coordinator's)
    store = dist.TCPStore(host, store_port, None, rank == 0, timeout=datetime.timedelta(seconds=300),
                          wait_for_workers=False)
    coord = None
    if rank == 0:
        coord = coordinator(host, control_port, ephemeral_ports=True, lease_s=lease_s, data_plane="p2p")
        store.set("vcx/node_job/coordinator", "up")
    else:
        store.wait(["vcx/node_job/coordinator"])
    me = client(host, host, control_port=control_port, my_port=0, engine=engine_factory(), out_dir=out_dir,
                out_ext=out_ext, chunk=chunk)
    me.preresize = preresize
    store.add("vcx/node_job/joined", 1)
    try:
        if rank != 0:
            while not store.check([DONE_KEY]):
                time.sleep(0.05)
            return int(me.metrics.counters.get("frames_processed", 0))
        t_join = time.time() + 300
        while int(store.add("vcx/node_job/joined", 0)) < world:  # every volunteer is in the pool
            if time.time() > t_join:
                raise TimeoutError(f"only {int(store.add('vcx/node_job/joined', 0))} of {world} volunteers joined")
            time.sleep(0.01)
        me.become_requester(source)
        t = me.wait_job(timeout=timeout_s)
        st = {"frames": me.final_sent_frame, "job_s": t, "chunks": int(me.metrics.counters.get("chunks_sent", 0)),
              "out": me.path_out, "coordinator": dict(coord.metrics.counters),
              "requester": dict(me.metrics.counters)}
        store.set(DONE_KEY, "1")
        return st
    finally:
        me.exit_threads()
        if coord is not None:
            while int(store.add("vcx/node_job/left", 0)) < world - 1:  # workers left before we close
                time.sleep(0.01)
            coord.exit_threads()
        else:
            store.add("vcx/node_job/left", 1)
