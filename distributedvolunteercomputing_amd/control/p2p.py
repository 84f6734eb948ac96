"""Peer-to-peer chunk data plane of the volunteer video job.

The reference relays every chunk through the coordinator: requester -> coordinator -> worker
-> coordinator -> requester, four host hops per chunk (/root/reference/server.py:48-62,73,89;
worker.py:157,164-178). On the p2p plane the coordinator only moves METADATA (which chunk goes
to which worker, leases, re-dispatch); the chunk bytes travel once from the requester's memory
to the worker's and the annotated chunk once back, over a **directional pair group** per
(sender, receiver) volunteer pair:

* RCCL (``ProcessGroupNCCL``, one rank per GPU) between GPU volunteers: the chunk goes
  requester GPU -> worker GPU over xGMI and never touches the host on either side;
* gloo between CPU volunteers (and in the CPU tests).

Pairs are created lazily, from the coordinator-hosted rendezvous store, by the two volunteers
involved only (no global generation: a dead or slow volunteer never blocks the others), and
each pair carries ONE direction so that a worker's result send and the requester's next chunk
send can never wait on each other across one ordered communicator. Every pair runs its
operations in order on its own thread, in the order the coordinator's instructions arrive
(per-volunteer FIFO outboxes: both ends see the same order), and tags them with the chunk id.
A pair whose peer the coordinator declares dead is aborted (its watch trips: RCCL
``ncclCommAbort``; a gloo wait is abandoned), so a transfer to a crashed worker never blocks
the requester's transfers to the others, and the re-dispatched chunk goes out on another pair.

A transfer that fails between two LIVE volunteers (a transport error, a timeout) kills only that
pair's communicator: the failing end bumps the pair's generation in the store
(``vcx/p2p/<src>><dst>/gen``, one compare-and-set, so both ends' failures bump it once), drops
the pair, and reports the failure to its caller (the volunteer then tells the coordinator, which
re-dispatches the chunk). Before every operation a pair compares its generation with the store's
and is rebuilt under the new name if it is behind, so the other end — whose own operation may
have completed before the failure — moves to the fresh communicator too instead of waiting on
the broken one.
"""
from __future__ import annotations

import queue
import threading
import time

import torch

from ..parallel.peer_group import PeerFailure, PeerGroup


def _device_key(dev: torch.device) -> str:
    """Host + physical device identity (PCI bus id), equal for two processes on one GPU. The
    host part is RCCL's own: ``NCCL_HOSTID`` when set (RCCL's duplicate-GPU check compares that
    host hash and the bus id, so processes with distinct host ids may share a card — the one-GPU
    rehearsal of scripts/rccl_rehearsal_launch.py), else the hostname."""
    import os
    import socket

    host = os.environ.get("NCCL_HOSTID") or socket.gethostname()
    if dev.type != "cuda":
        return f"{host}/cpu/{id(dev)}"  # CPU ends never share an RCCL device
    props = torch.cuda.get_device_properties(dev)
    bus = getattr(props, "pci_bus_id", None)
    ident = f"{getattr(props, 'pci_domain_id', 0)}:{bus}:{getattr(props, 'pci_device_id', 0)}" if bus is not None \
        else str(getattr(props, "uuid", dev.index))
    return f"{host}/{ident}"


class _PairWatch:
    """The ``watch`` protocol of PeerGroup guarded waits, tripped by a peer_dead notice or — polled
    at most every 50 ms from the waiting pair thread — by the other end moving the pair to a new
    generation (its side of the transfer failed: this side's pending operation never completes)."""

    def __init__(self, pid, moved=None):
        self.pid = pid
        self._ev = threading.Event()
        self._reason = ""
        self._moved = moved  # () -> bool: has the pair's generation advanced in the store?
        self._next_check = 0.0

    def tripped(self) -> bool:
        if not self._ev.is_set() and self._moved is not None and time.monotonic() >= self._next_check:
            self._next_check = time.monotonic() + 0.05
            try:
                if self._moved():
                    self.declare_abort("the other end moved the pair to a new generation")
            except Exception:  # noqa: BLE001 — store unreachable: leave it to the timeouts
                pass
        return self._ev.is_set()

    def abort_reason(self) -> str:
        return self._reason

    def declare_abort(self, reason: str):
        self._reason = reason
        self._ev.set()


class _Pair:
    def __init__(self, plane, src: int, dst: int):
        self.plane = plane
        self.src, self.dst = src, dst
        self.watch = _PairWatch(plane.vid)
        self.q: queue.Queue = queue.Queue()
        self.group = None
        self.dead = False
        self.gen = None  # generation of the current communicator (from the store)
        self._store = None
        self.thread = threading.Thread(target=self._loop, name=f"vcx-p2p-{src}>{dst}", daemon=True)
        self.thread.start()

    def _gen_key(self):
        return f"vcx/p2p/{self.src}>{self.dst}/gen"

    def _store_gen(self) -> int:
        return int(self._store.add(self._gen_key(), 0))

    def _drop_group(self):
        g, self.group = self.group, None
        if g is not None:
            try:
                g.abort()
            except Exception:  # noqa: BLE001
                pass

    def _failed(self):
        """This end saw the communicator fail: move the pair to the next generation (once)."""
        if self._store is not None and self.gen is not None:
            try:
                self._store.compare_set(self._gen_key(), str(self.gen), str(self.gen + 1))
            except Exception:  # noqa: BLE001
                pass
        self._drop_group()

    def _group(self):
        if self._store is None:
            # a store client of its own: a c10d TCPStore client serialises its blocking waits, so
            # one pair stuck rendezvousing with a dead peer would stall every other pair's connect
            self._store = self.plane.store_factory()
            self._store.add(self._gen_key(), 0)
        cur = self._store_gen()
        if self.group is not None and cur != self.gen:  # the other end failed and moved on
            self.plane.metrics_incr("p2p_pair_rebuilt")
            self._drop_group()
        if self.group is None:
            rank = 0 if self.plane.vid == self.src else 1
            store = self._store
            self.gen = cur
            self.watch = _PairWatch(self.plane.vid, moved=lambda g=cur: self._store_gen() != g)
            name = f"p2p/{self.src}>{self.dst}/g{cur}"
            # non-blocking handshake first: the communicator is built only once both ends are
            # known to be up, so a peer that never shows (crashed before its first transfer)
            # leaves no rendezvous blocked inside c10d — the wait below is abortable
            # the hello carries each end's backend and device identity. RCCL only when both ends
            # run it on DIFFERENT devices (it refuses two ranks on one GPU; a CPU volunteer speaks
            # gloo only); otherwise the pair uses gloo, GPU tensors staged through host memory
            me = f"{self.plane.backend}|{self.plane.device_key}"
            store.set(f"vcx/{name}/hello{rank}", me)
            other = f"vcx/{name}/hello{1 - rank}"
            while not store.check([other]):
                if self.watch.tripped():
                    raise PeerFailure(f"pair {name}: {self.watch.abort_reason()}")
                time.sleep(0.002)
            o_backend, _, o_dev = store.get(other).decode().partition("|")
            backend = "nccl" if self.plane.backend == o_backend == "nccl" and o_dev != self.plane.device_key else "gloo"
            if self.plane.backend == "nccl" and backend == "gloo":
                self.plane.metrics_incr("p2p_same_device_pairs" if o_dev == self.plane.device_key
                                        else "p2p_mixed_backend_pairs")
            self.plane.metrics_incr(f"p2p_pairs_{backend}")
            g = PeerGroup(store, rank, 2, backend, generation=name, device=self.plane.device,
                          timeout_s=self.plane.timeout_s, watch=self.watch)
            g.connect()
            self.group = g
        return self.group

    def _loop(self):
        while True:
            op = self.q.get()
            if op is None:
                return
            kind, payload, tag, cb = op
            if self.dead:
                res = PeerFailure(f"pair {self.src}>{self.dst} is dead")
            else:
                try:
                    g = self._group()
                    if self.plane.inject_failures > 0 and kind == "recv":  # fault-injection tests
                        self.plane.inject_failures -= 1
                        raise PeerFailure(f"pair {self.src}>{self.dst}: injected transfer failure")
                    if kind == "send":
                        g.send(payload, 1, tag)
                        res = None
                    else:
                        shape, dtype = payload
                        # a host pair plane on a GPU volunteer receives into pinned memory: the chunk's
                        # next hop (the worker's upload, the requester's GPU Y4M conversion) is then a DMA
                        # instead of a staged copy (torch's caching host allocator recycles the buffers)
                        pin = self.plane.device.type == "cpu" and self.plane.pin_host
                        res = torch.empty(shape, dtype=dtype, device=self.plane.device, pin_memory=pin)
                        g.recv(res, 0, tag)
                except Exception as e:  # noqa: BLE001 — PeerFailure or a transport error: this pair only
                    self.plane.metrics_incr("p2p_failed")
                    if self.plane.is_dead_peer(self.src, self.dst):
                        self.dead = True  # the other end is gone for good
                    else:
                        self._failed()  # a live peer: a new generation at the next operation
                    res = e
            try:
                cb(res)
            except Exception:  # noqa: BLE001 — a consumer's bug must not kill the pair thread
                self.plane.metrics_incr("p2p_callback_errors")

    def close(self):
        self.q.put(None)


class PairPlane:
    """Directional pair groups of one volunteer (id ``vid``) over a shared rendezvous store
    (``store_factory()`` returns a new client connection to it)."""

    def __init__(self, store_factory, vid: int, backend: str = "gloo", device=None, timeout_s: float = 60.0,
                 metrics=None):
        self.store_factory = store_factory  # -> a fresh client of the coordinator-hosted store
        self.vid = int(vid)
        self.backend = backend
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.timeout_s = timeout_s
        self.metrics = metrics
        self._pairs: dict[tuple[int, int], _Pair] = {}
        self._lock = threading.Lock()
        self.device_key = _device_key(self.device)
        self._dead: set[int] = set()  # volunteers the coordinator declared dead
        self.inject_failures = 0  # tests: make this many receives fail like a broken transport
        self.pin_host = torch.cuda.is_available()  # host receives land in pinned memory on a GPU volunteer

    def is_dead_peer(self, src: int, dst: int) -> bool:
        return src in self._dead or dst in self._dead

    def metrics_incr(self, name):
        if self.metrics is not None:
            self.metrics.incr(name)

    def _pair(self, src: int, dst: int) -> _Pair:
        with self._lock:
            p = self._pairs.get((src, dst))
            if p is None:
                p = self._pairs[(src, dst)] = _Pair(self, src, dst)
            return p

    def send(self, dst: int, tensor: torch.Tensor, tag: int, cb=None):
        """Queue `tensor` for volunteer `dst` (it must post the matching recv with this tag)."""
        t = tensor.contiguous()
        if t.device != self.device:
            t = t.to(self.device)
        self._pair(self.vid, dst).q.put(("send", t, int(tag) % (1 << 30), cb or (lambda _r: None)))

    def recv(self, src: int, shape, dtype, tag: int, cb):
        """Queue a receive from volunteer `src`; ``cb(tensor)`` on arrival, ``cb(exception)`` on failure."""
        self._pair(src, self.vid).q.put(("recv", (tuple(shape), dtype), int(tag) % (1 << 30), cb))

    def peer_dead(self, vid: int):
        """The coordinator declared `vid` dead: abort every pair with it (in-flight ops fail fast)."""
        with self._lock:
            self._dead.add(int(vid))
            pairs = [p for (s, d), p in self._pairs.items() if vid in (s, d)]
        for p in pairs:
            p.dead = True
            p.watch.declare_abort(f"volunteer {vid} declared dead by the coordinator")

    def close(self):
        with self._lock:
            pairs = list(self._pairs.values())
            self._pairs.clear()
        for p in pairs:
            p.watch.declare_abort("plane closed")
            p.close()
        # release the pair communicators now, from this thread, once their pair threads are done:
        # a gloo process group left to interpreter finalisation aborts the process in its
        # destructor ("terminate called without an active exception")
        for p in pairs:
            p.thread.join(timeout=5.0)
            if not p.thread.is_alive() and p.group is not None:
                g, p.group = p.group, None
                if g.backend == "nccl":
                    g.shutdown()
                g.pg = None
