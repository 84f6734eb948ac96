"""The coordinator: membership, data-port allocation, chunk dispatch, result routing.

Public API kept from the reference (/root/reference/server.py):
``coordinator(ip='localhost')``, ``.exit_threads()``, ``.log(msg)``, class-level tunables
``verbose``, ``req_rep``, ``max_buffer`` and the 5555..5599 data-port pool; the UDP verbs
join/request/stop/end with ``ok||<port>`` / ``ok`` replies.

What happens where:
* UDP control thread (``manager``)      — reference C4, plus ``hb``/``status`` verbs.
* one ingest thread per volunteer       — reference C5: a ``FrameHub`` on that volunteer's port;
  ``request`` chunks go to the scheduler, ``processed`` chunks to the requester's router.
* dispatcher thread                     — reference C6, but the policy/ledger is the C++
  ``ChunkScheduler``: no dropped chunks, requester exclusion, per-worker credits, re-dispatch.
* one outbox thread per volunteer       — owns that volunteer's ``FrameSender``; both dispatched
  work and routed results go through it, so a socket is never used by two threads
  (the reference shares one REQ socket between two threads).
* lease monitor                         — expires silent volunteers, re-queues their chunks.

Data planes (``data_plane=``): ``relay`` moves chunk bytes through this process like the
reference (host TCP, for CPU-only volunteers); ``p2p`` moves only metadata through it — chunks go
requester -> worker and back over directional pair groups (control/p2p.py: RCCL over xGMI between
GPU volunteers), the coordinator tells both ends of each transfer when to post it, keeps the
leases and re-dispatches a dead worker's chunks exactly as on the relay plane.

All mutable state is per instance (the reference keeps it in class attributes shared by every
instance, server.py:13-24).
"""
from __future__ import annotations

import itertools
import json
import queue
import secrets
import socket
import threading
import time
from collections import deque

import numpy as np

from .. import _native_loader
from ..utils.metrics import Metrics
from . import protocol
from .transport import BadFrame, FrameHub, FrameSender


_EMPTY = np.zeros(0, dtype=np.uint8)  # payload of a metadata-only frame


def _window(w):
    """A well-formed shared-source window {path: str, first: int >= 0, n: int > 0}, else None (the chunk
    then travels as frames). Only the shape is checked here; each worker checks the path against its own
    shared_source_root before it reads anything (peer._read_window)."""
    if not isinstance(w, dict):
        return None
    path, first, n = w.get("path"), w.get("first"), w.get("n")
    if not isinstance(path, str) or not path or len(path) > 4096:
        return None
    if not all(isinstance(x, int) and not isinstance(x, bool) for x in (first, n)) or first < 0 or n <= 0:
        return None
    return {"path": path, "first": first, "n": n}


class _Volunteer:
    def __init__(self, addr, port, hub, sender, vid=0):
        self.vid = vid
        self.addr = addr
        self.port = port
        self.hub = hub
        self.sender = sender
        self.outbox: queue.Queue = queue.Queue()
        self.alive = True
        self.threads: list[threading.Thread] = []


class coordinator:  # noqa: N801  (reference class name)
    verbose = False
    req_rep = True
    max_buffer = 40
    port_pool = tuple(range(5555, 5600))
    lease_s = 10.0

    def log(self, message):
        if self.verbose:
            print(message, flush=True)

    def __init__(self, ip: str = "localhost", control_port: int = protocol.DEFAULT_CONTROL_PORT, *,
                 ephemeral_ports: bool = False, max_clients: int | None = None, policy: str = "round_robin",
                 credits: int = 2, lease_s: float | None = None, verbose: bool | None = None,
                 train_store_port: int | None = None, data_plane: str = "relay", train_token: str | None = None):
        if verbose is not None:
            self.verbose = verbose
        if data_plane not in ("relay", "p2p"):
            raise ValueError(f"data_plane must be 'relay' or 'p2p', not {data_plane!r}")
        self.data_plane = data_plane
        if data_plane == "p2p" and train_store_port is None:
            train_store_port = 0  # the pair groups rendezvous on this process's store
        # Rendezvous store for training peers (heartbeats, generations, RCCL bootstrap). Hosted
        # here so that ANY training peer may die without taking the membership state with it.
        # Access control: torch's TCPStore listens on every interface and has no authentication,
        # so every key the peers use lives under a per-coordinator random prefix (`store_secret`)
        # that is handed out only to admitted training peers (`tjoin`, optionally gated by
        # `train_token`) and, in a job without a token, to joined volunteers (the `store` verb); the
        # `store` verb is refused to anyone else. A host that can reach the port but never joined cannot name, so cannot forge, the
        # abort / join / pair-hello records the peers act on (the reference binds every interface
        # with no auth at all: /root/reference/server.py:96).
        # Two prefixes: `store_secret` (the training membership keys) and `p2p_secret` (the chunk
        # plane's pair-group rendezvous). A joined volunteer only ever learns the p2p one; with a
        # `train_token` the training prefix goes out only through an admitted `tjoin`, so joining
        # as a volunteer (unauthenticated, any host) gives no way to read or forge training keys.
        self.store_secret = secrets.token_hex(16)
        self.p2p_secret = secrets.token_hex(16)
        self.train_token = train_token
        self.train_peers: set[str] = set()
        self.train_store = None
        if train_store_port is not None:
            import datetime

            import torch.distributed as dist

            self.train_store = dist.TCPStore("0.0.0.0", int(train_store_port), None, True,
                                             timeout=datetime.timedelta(seconds=300), wait_for_workers=False)
            self.train_store_port = self.train_store.port
        if lease_s is not None:
            self.lease_s = lease_s
        N = _native_loader.native()
        pol = N.ChunkScheduler.Policy.LEAST_LOADED if policy == "least_loaded" else N.ChunkScheduler.Policy.ROUND_ROBIN
        self.sched = N.ChunkScheduler(int(pol), credits)
        self.ephemeral = ephemeral_ports
        nports = max_clients or len(self.port_pool)
        self.free_ports = deque([0] * nports if ephemeral_ports else list(self.port_pool)[:nports])
        self.vols: dict[str, _Volunteer] = {}
        self.port_to_client: dict[int, str] = {}
        self.chunks: dict[int, tuple] = {}
        self.requesters: set[str] = set()
        self.peer_metrics: dict[str, dict] = {}  # volunteer -> its last metrics report
        self._ids = itertools.count(1)
        self._vids = itertools.count(1)
        self._lock = threading.RLock()
        self._work = threading.Condition()
        self.metrics = Metrics("coordinator")
        self.continue_listening = True
        self.continue_send_request = True

        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind(("", int(control_port)))
        self.sock.settimeout(0.25)
        self.control_port = self.sock.getsockname()[1]
        self.my_ip = f"{ip}:{self.control_port}"
        self._threads = [
            threading.Thread(target=self.manager, name="vcx-manager", daemon=True),
            threading.Thread(target=self.send_request, name="vcx-dispatch", daemon=True),
            threading.Thread(target=self._lease_monitor, name="vcx-lease", daemon=True),
        ]
        for t in self._threads:
            t.start()
        self.log(f"listening on {self.my_ip}")

    # ------------------------------------------------------------------ control plane
    def manager(self):
        while self.continue_listening:
            try:
                data, src = self.sock.recvfrom(4096)
            except socket.timeout:
                continue
            except OSError:
                break
            verb, addr = protocol.decode(data)
            if verb is None:
                continue
            try:
                reply = self._handle(verb, addr, src)
            except Exception as e:  # never let one bad datagram kill the control loop
                reply = f"err{protocol.SEP}{e}".encode()
            if reply is not None:
                try:
                    self.sock.sendto(reply, src)
                except OSError:
                    pass
        self.log("manager terminated.")

    def _handle(self, verb, addr, src=None):
        now = time.time()
        if verb == "join":
            if src is not None and not protocol.addr_matches(addr, src[0]):
                self.metrics.incr("spoofed_datagrams")
                return f"err{protocol.SEP}address {addr} does not match sender {src[0]}".encode()
            return self._join(addr, now)
        if verb == "tjoin":  # a training peer asks for the rendezvous store
            return self._tjoin(addr, src)
        if verb in ("request", "stop", "end", "hb", "p2p", "store"):
            with self._lock:
                if verb == "store" and self.train_token is not None:
                    known = addr in self.train_peers  # token-gated job: admitted training peers only
                else:
                    known = addr in self.vols or (verb == "store" and addr in self.train_peers)
            if not known or (src is not None and not protocol.addr_matches(addr, src[0])):
                self.metrics.incr("unknown_datagrams")
                return f"err{protocol.SEP}{addr} has not joined".encode()
        if verb == "request":
            self.sched.set_available(addr, False)
            with self._lock:
                self.requesters.add(addr)
            self.metrics.incr("requests")
            return protocol.reply_ok()
        if verb == "stop":
            self.sched.set_available(addr, True)
            self._kick()
            return protocol.reply_ok()
        if verb == "end":
            self._remove(addr, reason="end")
            return protocol.reply_ok()
        if verb == "hb":
            self.sched.heartbeat(addr, now)
            return protocol.reply_ok()
        if verb == "status":
            st = self.status()
            js = json.dumps(st)
            if len(js) > 60000:  # one UDP datagram: per-volunteer details give way to the totals
                st["peers"]["volunteers"] = {a: {"truncated": True} for a in st["peers"]["volunteers"]}
                js = json.dumps(st)
            return protocol.reply_ok(js)
        if verb == "store":  # where training peers rendezvous (joined volunteers / admitted peers only)
            return protocol.reply_ok(self._store_ref())
        if verb == "p2p":
            with self._lock:
                v = self.vols.get(addr)
            info = {"plane": self.data_plane, "vid": v.vid if v is not None else None,
                    "store_port": self.train_store_port if self.data_plane == "p2p" else None,
                    "store_prefix": self.p2p_secret if self.data_plane == "p2p" else None}
            return protocol.reply_ok(json.dumps(info))
        return None

    def _store_ref(self) -> str:
        """`<port>||<key prefix>` of the rendezvous store ('' when this coordinator hosts none)."""
        if self.train_store is None:
            return ""
        return f"{self.train_store_port}{protocol.SEP}{self.store_secret}"

    def _join_reply(self, port) -> bytes:
        # `ok||<port>` as in the reference; with a rendezvous store a third field carries the p2p
        # plane's key prefix (the reference client reads only field 1: worker.py:61). Never the
        # training prefix: `join` is unauthenticated.
        if self.train_store is None:
            return protocol.reply_ok(str(port))
        return protocol.reply_ok(f"{port}{protocol.SEP}{self.p2p_secret}")

    def _tjoin(self, addr, src):
        """Admit a training peer `<id>[||<token>]`: reply `ok||<store port>||<key prefix>`."""
        ident, _, token = addr.partition(protocol.SEP)
        if self.train_store is None:
            return f"err{protocol.SEP}this coordinator hosts no rendezvous store".encode()
        if self.train_token is not None and not secrets.compare_digest(token, self.train_token):
            self.metrics.incr("refused_tjoin")
            return f"err{protocol.SEP}bad admission token".encode()
        with self._lock:
            self.train_peers.add(ident)
        self.metrics.incr("train_peers")
        return protocol.reply_ok(self._store_ref())

    def _join(self, addr, now):
        with self._lock:
            v = self.vols.get(addr)
            if v is not None:  # idempotent re-join (lost ack): same port, no duplicate
                self.sched.add_worker(addr, now)
                return self._join_reply(v.port)
            if not self.free_ports:
                return f"err{protocol.SEP}no free data port".encode()
            port = self.free_ports.popleft()
            hub = FrameHub(port, REQ_REP=self.req_rep, capacity=max(2, self.max_buffer))
            port = hub.port
            host, cport = protocol.split_addr(addr)
            try:
                sender = FrameSender(f"tcp://{host}:{cport}", REQ_REP=self.req_rep, connect_timeout=5.0)
            except Exception:
                hub.close()
                self.free_ports.appendleft(0 if self.ephemeral else port)
                raise
            v = _Volunteer(addr, port, hub, sender, vid=next(self._vids))
            self.vols[addr] = v
            self.port_to_client[port] = addr
            for fn, nm in ((self._ingest, "ingest"), (self._outbox, "outbox")):
                t = threading.Thread(target=fn, args=(v,), name=f"vcx-{nm}-{addr}", daemon=True)
                v.threads.append(t)
                t.start()
            self.sched.add_worker(addr, now)
            self.metrics.incr("joins")
            self.log(f"join {addr} -> data port {port}")
        self._kick()
        return self._join_reply(port)

    def _remove(self, addr, reason):
        with self._lock:
            v = self.vols.pop(addr, None)
            self.requesters.discard(addr)
            self.peer_metrics.pop(addr, None)
        requeued = self.sched.remove_worker(addr)
        if v is not None:
            self.metrics.incr("leaves_" + reason)
        self.metrics.counters["redispatched"] = self.sched.requeued  # by removal and by lease expiry
        dropped = self.sched.cancel_requester(addr)
        if dropped:  # its queued chunks will never be dispatched: free their frames
            with self._lock:
                for cid in dropped:
                    self.chunks.pop(cid, None)
            self.metrics.incr("chunks_cancelled", len(dropped))
        if v is None:
            return
        v.alive = False
        if self.data_plane == "p2p":  # every other volunteer aborts its pair groups with this one
            with self._lock:
                others = list(self.vols.values())
            for o in others:
                o.outbox.put(("coordinator||peer_dead", _EMPTY, {"p2p": 1, "cmd": "peer_dead", "vid": v.vid}))
        self.port_to_client.pop(v.port, None)
        self.free_ports.append(0 if self.ephemeral else v.port)
        v.outbox.put(None)
        v.hub.close()
        v.sender.close()
        if requeued:
            self.log(f"{addr} left ({reason}); re-queued chunks {requeued}")
        self._kick()

    def _lease_monitor(self):
        while self.continue_listening:
            time.sleep(max(0.05, self.lease_s / 4))
            for addr in self.sched.expire(time.time(), self.lease_s):  # drops them, re-queues their chunks
                self.log(f"lease expired: {addr}")
                self._remove(addr, reason="lease")

    # ------------------------------------------------------------------ data plane
    def _ingest(self, v: _Volunteer):
        while v.alive and self.continue_listening:
            try:
                r = v.hub.recv_frame(timeout=0.25)
            except BadFrame as e:  # a malformed frame costs its sender the frame, not the thread
                self.metrics.incr("bad_frames")
                self.log(f"bad frame from {v.addr}: {e}")
                continue
            if r is None:
                continue
            hdr, arr, _ = r
            self.sched.heartbeat(v.addr, time.time())
            info = hdr.get("msg", "")
            parts = info.split(protocol.SEP)
            if len(parts) < 2:
                continue
            requester, command = parts[0], parts[1]
            p2p = bool(hdr.get("p2p"))
            if command == "metrics":  # a volunteer's metrics report: kept per volunteer
                m = hdr.get("metrics")
                if isinstance(m, dict):
                    with self._lock:
                        self.peer_metrics[v.addr] = m
                continue
            if p2p and command in ("request", "processed") and not protocol.valid_chunk_shape(hdr.get("cshape")):
                self.metrics.incr("bad_frames")  # a shape the other end would have to allocate blindly
                continue
            if command == "failed" and p2p:  # a pair transfer of this chunk to v failed
                cid = int(hdr.get("chunk", -1))
                if hdr.get("nowin"):  # v cannot read the chunk's shared-source window: the requester sends it
                    with self._lock:
                        rec = self.chunks.get(cid)
                        if rec is not None and rec[2] is not None:
                            rec[2]["win"] = None
                    self.metrics.incr("window_fallbacks")
                if self.sched.fail(cid, v.addr):
                    self.metrics.incr("p2p_failed_requeued")
                    self._kick()
                continue
            if command == "request":
                while self.req_rep and self.sched.queued() > self.max_buffer and v.alive:
                    time.sleep(0.005)  # back-pressure: the hub stops acking, TCP throttles the requester
                cid = next(self._ids)
                with self._lock:
                    # p2p: metadata only — the frames stay in the requester's (GPU) memory
                    # shared-source mode: `win` = the chunk's index window in a file the workers read themselves
                    self.chunks[cid] = (info, None, {"key": hdr.get("key"), "cshape": hdr.get("cshape"),
                                                     "src": v.vid, "win": _window(hdr.get("win"))}) if p2p \
                        else (info, arr, None)
                self.sched.submit(cid, requester)
                self.metrics.incr("chunks_in")
                self._kick()
            elif command == "processed":
                cid = int(hdr.get("chunk", -1))
                if not self.sched.complete(cid):
                    self.metrics.incr("duplicate_results")
                    if p2p:  # the worker holds the duplicate result: let it free it
                        v.outbox.put((info, _EMPTY, {"p2p": 1, "cmd": "drop", "chunk": cid}))
                    continue  # late duplicate of a re-dispatched chunk
                with self._lock:
                    rec = self.chunks.pop(cid, None)
                    dst = self.vols.get(requester)
                if dst is not None:
                    if p2p:  # both ends post the transfer of the result: worker -> requester
                        key = rec[2]["key"] if rec is not None and rec[2] else None
                        v.outbox.put((info, _EMPTY, {"p2p": 1, "cmd": "send_result", "chunk": cid, "dst": dst.vid,
                                                     "cshape": hdr.get("cshape")}))
                        dst.outbox.put((info, _EMPTY, {"p2p": 1, "cmd": "recv_result", "chunk": cid, "src": v.vid,
                                                       "cshape": hdr.get("cshape"), "key": key}))
                    else:
                        dst.outbox.put((info, arr, {"chunk": cid}))
                elif p2p:
                    v.outbox.put((info, _EMPTY, {"p2p": 1, "cmd": "drop", "chunk": cid}))
                self.metrics.incr("chunks_done")
                self._kick()

    def _outbox(self, v: _Volunteer):
        while v.alive:
            item = v.outbox.get()
            if item is None:
                break
            info, arr, meta = item
            ok = v.sender.send_image(info, arr, **meta)
            if not ok:
                self.log(f"send to {v.addr} failed; removing")
                self._remove(v.addr, reason="broken")
                break

    def _kick(self):
        with self._work:
            self._work.notify_all()

    def send_request(self):
        """Dispatcher (reference C6): FIFO chunks -> eligible volunteers (never dropped)."""
        while self.continue_send_request:
            a = self.sched.next()
            if not a.valid():
                with self._work:
                    self._work.wait(timeout=0.05)
                continue
            with self._lock:
                item = self.chunks.get(a.chunk)
                v = self.vols.get(a.worker)
                r = self.vols.get(a.requester)
            if item is None:
                self.sched.complete(a.chunk)
                continue
            if v is None:
                self.sched.requeue_front(a.chunk, a.requester)
                continue
            info, arr, meta = item
            if meta is None:
                v.outbox.put((info, arr, {"chunk": a.chunk}))
            elif r is None:  # the requester left: nobody holds the frames any more
                self.sched.complete(a.chunk)
                with self._lock:
                    self.chunks.pop(a.chunk, None)
                continue
            elif meta.get("win") is not None:  # shared source: the worker reads the window itself
                v.outbox.put((info, _EMPTY, {"p2p": 1, "cmd": "work", "chunk": a.chunk, "src": meta["src"],
                                             "cshape": meta["cshape"], "key": meta["key"], "win": meta["win"]}))
                self.metrics.incr("window_dispatched")
            else:  # p2p: the worker posts the receive, the requester the send, of the same chunk
                v.outbox.put((info, _EMPTY, {"p2p": 1, "cmd": "work", "chunk": a.chunk, "src": meta["src"],
                                             "cshape": meta["cshape"], "key": meta["key"]}))
                r.outbox.put((info, _EMPTY, {"p2p": 1, "cmd": "send", "chunk": a.chunk, "dst": v.vid,
                                             "key": meta["key"], "cshape": meta["cshape"]}))
            self.metrics.incr("dispatched")
        self.log("send_request terminated.")

    # ------------------------------------------------------------------ misc
    def status(self) -> dict:
        return {
            "workers": self.sched.workers(),
            "available": self.sched.available_workers(),
            "queued": self.sched.queued(),
            "inflight": self.sched.inflight(),
            "dispatched": self.sched.dispatched,
            "free_ports": len(self.free_ports),
            "data_plane": self.data_plane,
            "metrics": self.metrics.snapshot(),
            "peers": self.peer_report(),
        }

    def peer_report(self) -> dict:
        """Per-volunteer metrics (last report of each live volunteer) and their counter totals."""
        with self._lock:
            per = {a: m for a, m in self.peer_metrics.items() if a in self.vols}
        totals: dict[str, float] = {}
        for m in per.values():
            for k, val in (m.get("counters") or {}).items():
                if isinstance(val, (int, float)):
                    totals[k] = totals.get(k, 0) + val
        return {"volunteers": per, "totals": totals}

    @property
    def clients(self):
        """The available worker pool (reference attribute name)."""
        return self.sched.available_workers()

    def exit_threads(self):
        self.continue_listening = False
        self.continue_send_request = False
        self._kick()
        for addr in list(self.vols):
            self._remove(addr, reason="shutdown")
        for t in self._threads:
            t.join(timeout=2)
        try:
            self.sock.close()
        except OSError:
            pass


Coordinator = coordinator
