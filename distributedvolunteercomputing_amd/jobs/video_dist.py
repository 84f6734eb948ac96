"""The video job over the RCCL/xGMI data plane.

On one 8×MI355X node every volunteer is a GPU process. Instead of the reference's star
(requester -> coordinator -> worker -> coordinator -> requester: four host hops per chunk,
/root/reference/server.py:57-89), chunks move GPU-to-GPU over xGMI with point-to-point
sends of the peer group, and the coordinator only sees metadata:

  requester: host decode -> pinned H2D -> batched resize to 400 px (HIP) -> send(chunk) to
             worker k mod P  ...  recv(annotated chunk) -> D2H -> in-order sink
  worker   : recv(chunk) into its HBM -> preprocess + MobileNet-SSD + NMS + annotate (HIP)
             -> send(annotated chunk) back

A chunk message is an int64 header [chunk_id, n, h, w, first_frame, 0, 0, 0] followed by the
uint8 [n, h, w, 3] payload (sizes must be known before a receive is posted). Work goes out in
rounds of one chunk per worker (credit 1 per worker keeps blocking point-to-point on a single
RCCL stream deadlock-free); the requester decodes the next round on a host thread while the
workers compute. chunk_id = -1 terminates a worker.
"""
from __future__ import annotations

import queue
import threading
import time

import numpy as np
import torch

from ..io.video import open_sink, open_source
from ..ops import vision as V
from .video import Engine, OrderedSink

HDR = 8


def _hdr(dev, *vals):
    h = torch.zeros(HDR, dtype=torch.int64)
    h[: len(vals)] = torch.tensor(vals, dtype=torch.int64)
    return h.to(dev)


def run_worker(group, engine: Engine, device, requester_rank: int = 0, requester_name: str = "requester"):
    """Serve chunks from the requester until the terminate header arrives."""
    hdr = torch.zeros(HDR, dtype=torch.int64, device=device)
    served = 0
    while True:
        group.recv(hdr, requester_rank, tag=1)
        cid, n, h, w = (int(v) for v in hdr[:4].tolist())
        if cid < 0:
            return served
        buf = torch.empty((n, h, w, 3), dtype=torch.uint8, device=device)
        group.recv(buf, requester_rank, tag=2)
        out = engine.process_tensor(buf, requester_name).contiguous()
        group.send(_hdr(device, cid, out.shape[0], out.shape[1], out.shape[2], int(hdr[4])), requester_rank, tag=3)
        group.send(out, requester_rank, tag=4)
        served += 1


def run_requester(group, source: str, out_path: str, device, *, chunk: int = 100, width: int = 400,
                  engine: Engine | None = None, fps: int = 30):
    """Stream `source` through the workers of `group` (every rank but this one). Returns stats.
    With no other peer the requester processes its chunks itself (engine required)."""
    me = group.rank if group is not None else 0
    workers = [r for r in range(group.size if group is not None else 1) if r != me]
    src = open_source(source)
    sink = OrderedSink(lambda w_, h_: open_sink(out_path, w_, h_, fps))
    chunks: queue.Queue = queue.Queue(maxsize=2 * max(1, len(workers)))

    def reader():  # host decode on its own thread, overlapped with the GPU round
        n, frames = 0, []
        while True:
            ok, f = src.read()
            if ok:
                frames.append(f)
            if frames and (not ok or len(frames) == chunk):
                chunks.put((n + 1, np.stack(frames)))
                n += len(frames)
                frames = []
            if not ok:
                chunks.put(None)
                return

    th = threading.Thread(target=reader, daemon=True)
    th.start()
    t0 = time.time()
    cid = 0
    total = 0
    done = False
    while not done:
        round_ = []
        for w in workers or [None]:
            item = chunks.get()
            if item is None:
                done = True
                break
            first, frames = item
            x = torch.from_numpy(frames).to(device, non_blocking=True)
            if x.shape[2] != width:
                x = V.resize_width(x, width).contiguous()
            if w is None:
                out = engine.process_tensor(x, "requester")
                round_.append((None, first, out))
            else:
                group.send(_hdr(device, cid, x.shape[0], x.shape[1], x.shape[2], first), w, tag=1)
                group.send(x, w, tag=2)
                round_.append((w, first, None))
            cid += 1
        for w, first, out in round_:
            if w is not None:
                hdr = torch.zeros(HDR, dtype=torch.int64, device=device)
                group.recv(hdr, w, tag=3)
                n, h, wd = (int(v) for v in hdr[1:4].tolist())
                out = torch.empty((n, h, wd, 3), dtype=torch.uint8, device=device)
                group.recv(out, w, tag=4)
            host = out.cpu().numpy()
            for i in range(host.shape[0]):
                sink.push(first + i, host[i])
            total += host.shape[0]
    for w in workers:
        group.send(_hdr(device, -1, 0, 0, 0, 0), w, tag=1)
    sink.set_final(total)
    th.join(timeout=5)
    dt = time.time() - t0
    print(f"final frame time taken for the job = {dt}", flush=True)
    return {"frames": total, "job_s": dt, "fps": total / dt if dt > 0 else None, "chunks": cid,
            "workers": len(workers)}
