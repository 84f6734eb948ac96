"""A group of volunteer peers that can be rebuilt on membership change — and abandoned
mid-collective when one of them dies.

Each generation of the training membership gets its OWN raw c10d process group, created
directly from a (prefixed) store with ``ProcessGroupNCCL`` (RCCL on ROCm, over xGMI) or
``ProcessGroupGloo`` (CPU volunteers / tests). Unlike ``dist.new_group`` this does not need
every member of the *previous* generation to take part, so survivors can re-form a group
after a peer has died (SURVEY.md §5.3 "(N) dropout-tolerant averaging").

Guarded collectives. When a ``watch`` (the elastic membership) is attached, no collective is
waited on blindly: the issuing thread polls ``work.is_completed()`` and the watch's abort flag.
The watch's heartbeat thread trips that flag when a member's lease expires while a collective
is in flight, or when another member posted an abort for this generation; the waiting peer
then aborts its communicator (``ProcessGroupNCCL.abort()`` = ``ncclCommAbort``: the RCCL
kernels spinning on the dead peer's xGMI link exit) and raises ``PeerFailure``. Gloo cannot
cancel an in-flight op (its ``abort`` returns but the pending pair read stays), so an aborted
gloo group is parked in ``_GRAVEYARD`` (never destroyed: its destructor would join the blocked
worker thread) and its buffers are abandoned by the caller.

Reference analog: the coordinator's ``clients`` pool mutated by join/end verbs
(/root/reference/server.py:104-154) — here the pool is a generation-numbered member list — and
the blocking send to a dead volunteer that stalls the reference's dispatcher forever
(/root/reference/server.py:89), which the guarded wait replaces.
"""
from __future__ import annotations

import datetime as _dt
import threading
import time

import torch
import torch.distributed as dist

from .. import config


class PeerFailure(RuntimeError):
    """A collective of this generation cannot complete: a member died, stopped or aborted."""


_GRAVEYARD: list = []  # aborted gloo groups with possibly blocked ops (see module docstring)
_ABORTING: list = []  # (RCCL group, thread running its ncclCommAbort): kept alive until it returns


def _abort_quietly(pg):
    try:
        pg.abort()
    except Exception:  # noqa: BLE001
        pass


def _gloo_pg(store, rank, size, timeout):
    opts = dist.ProcessGroupGloo._Options()
    opts._timeout = timeout
    host = config.get().gloo_host
    opts._devices = [dist.ProcessGroupGloo.create_device(hostname=host)]
    return dist.ProcessGroupGloo(store, rank, size, opts)


def _nccl_pg(store, rank, size, timeout):
    opts = dist.ProcessGroupNCCL.Options()
    opts._timeout = timeout
    return dist.ProcessGroupNCCL(store, rank, size, opts)


class PeerGroup:
    """One generation of live peers: rank/size are positions in ``members``."""

    def __init__(self, store, rank: int, size: int, backend: str = "gloo", *, generation: int = 0,
                 members=None, timeout_s: float = 300.0, device=None, watch=None):
        self.generation = generation
        self.members = list(members) if members is not None else list(range(size))
        self.rank = rank
        self.size = size
        self.backend = backend
        self.device = device
        self.watch = watch  # ElasticMembership (or None: plain blocking collectives)
        self.aborted = False
        self._abort_lock = threading.Lock()  # abort() may race between the watchdog and the waiter
        self.fault_hook = None  # test hook: called inside every guarded collective (after issue)
        self.poll_s = 2e-4
        self._pending = None  # deferred gloo rendezvous (watched groups connect in connect())
        self._connected = False
        self._bg = None  # (thread, result box) of a communicator build started by start_connect()
        self.bg_build_ms = None  # how long that build ran (staged admission)
        self.needs_go = False  # first guarded collective waits for every continuing member (elastic)
        timeout = _dt.timedelta(seconds=timeout_s)
        prefixed = dist.PrefixStore(f"vcx/pg/{generation}", store)
        self.pg = None
        if size == 1:
            pass
        elif backend == "nccl":
            self.pg = _nccl_pg(prefixed, rank, size, timeout)
        elif backend == "gloo":
            if watch is None:
                self.pg = _gloo_pg(prefixed, rank, size, timeout)
            else:  # the full-mesh connect blocks until every member shows up: make it abortable
                self._pending = (prefixed, rank, size, timeout)
        else:
            raise ValueError(f"unknown backend {backend!r}")

    @classmethod
    def from_default(cls, device=None) -> "PeerGroup":
        """Wrap torch.distributed's default process group (e.g. the torchrun world)."""
        self = cls.__new__(cls)
        self._pending = None
        self._bg = None
        self.bg_build_ms = None
        self.needs_go = False
        self._connected = True  # the default group is connected by init_process_group
        self.generation = 0
        self.size = dist.get_world_size()
        self.rank = dist.get_rank()
        self.members = list(range(self.size))
        self.backend = dist.get_backend()
        self.device = device
        self.watch = None
        self.aborted = False
        self._abort_lock = threading.Lock()
        self.fault_hook = None
        self.poll_s = 2e-4
        self.pg = dist.distributed_c10d._get_default_group() if self.size > 1 else None
        return self

    def connect(self):
        """Create the RCCL communicator now, bound to this peer's GPU (every member calls this
        right after adopting the generation, with the watchdog armed), instead of lazily inside
        the first collective. With ``TORCH_NCCL_USE_COMM_NONBLOCKING=1`` (set by the elastic
        membership) the init is non-blocking, so a member dying during it is aborted like any
        collective. No-op for gloo (connected in the constructor). A build started earlier by
        ``start_connect`` is joined here (abortable like the gloo rendezvous)."""
        if self._bg is not None:
            self._join_bg()
            return
        if self._pending is not None:
            self._connect_gloo()
            return
        if self.pg is None or self.backend != "nccl" or self.device is None or self._connected:
            return
        dev = torch.device(self.device)
        if dev.type == "cuda":
            self._check()
            # once per generation: ProcessGroupNCCL.eager_connect_single_device builds a NEW
            # communicator on every call (a second bootstrap per round, whose ranks can pick up
            # different unique ids and hang the next collective)
            self.pg.eager_connect_single_device(dev)
            self._connected = True

    def start_connect(self):
        """Start building this generation's communicator and return at once (staged admission: the
        members of the current generation build the next one -- which adds the joiners -- during
        their local steps, so the admission round itself pays no communicator init). RCCL: a
        non-blocking init issued here; gloo: the full-mesh rendezvous on a helper thread. Construct
        such a group on a store client of its own: a TCPStore client serialises the requests of all
        its threads, and the bootstrap must not queue behind the training thread's waits."""
        if self._bg is not None or self._connected or self.size == 1:
            return
        if self._pending is not None:
            args, self._pending = self._pending, None

            def build(box):
                box["pg"] = _gloo_pg(*args)
        elif self.pg is not None and self.backend == "nccl" and self.device is not None \
                and torch.device(self.device).type == "cuda":
            # on the calling thread: with TORCH_NCCL_USE_COMM_NONBLOCKING=1 (set by the elastic
            # membership) ncclCommInitRankConfig returns at once (measured 1 ms at 8 ranks) and RCCL
            # finishes the init on its own thread while this process keeps stepping; the first
            # collective waits for it. (A Python helper thread driving the init while the training
            # thread ran another communicator's all-to-all crashed every member, SIGSEGV, at 8 ranks.)
            t0 = time.perf_counter()
            self.pg.eager_connect_single_device(torch.device(self.device))
            self.bg_build_ms = (time.perf_counter() - t0) * 1e3
            self._connected = True
            return
        else:
            return
        box = {}

        def run():
            t0 = time.perf_counter()
            try:
                build(box)
            except Exception as e:  # noqa: BLE001
                box["err"] = e
            box["ms"] = (time.perf_counter() - t0) * 1e3

        th = threading.Thread(target=run, name=f"vcx-pg{self.generation}-build", daemon=True)
        th.start()
        self._bg = (th, box)

    def _join_bg(self):
        th, box = self._bg
        while th.is_alive():
            if self.watch is not None and self.watch.tripped():
                self._bg = None
                if self.backend == "nccl":
                    self.abort()
                self.aborted = True
                raise PeerFailure(f"gen {self.generation}: connect aborted ({self.watch.abort_reason()})")
            th.join(0.005)
        self._bg = None
        self.bg_build_ms = box.get("ms")
        if "err" in box:
            if self.watch is not None:
                self.watch.declare_abort(f"gen {self.generation} connect failed on peer {self.watch.pid}: {box['err']}")
            self.aborted = True
            raise PeerFailure(f"gen {self.generation}: connect failed: {box['err']}")
        if "pg" in box:
            self.pg = box["pg"]
        self._connected = True
        if self.aborted:  # the watchdog aborted us while the build was finishing
            pg, self.pg = self.pg, None
            if pg is not None and self.backend == "gloo":
                _GRAVEYARD.append(pg)
            raise PeerFailure(f"gen {self.generation}: aborted during connect")

    def _connect_gloo(self):
        args, self._pending = self._pending, None
        box = {}

        def build():
            try:
                box["pg"] = _gloo_pg(*args)
            except Exception as e:  # noqa: BLE001
                box["err"] = e

        th = threading.Thread(target=build, name=f"vcx-pg{self.generation}-connect", daemon=True)
        th.start()
        while th.is_alive():
            if self.watch.tripped():
                self.aborted = True
                raise PeerFailure(f"gen {self.generation}: connect aborted ({self.watch.abort_reason()})")
            th.join(0.01)
        if "err" in box:
            self.watch.declare_abort(f"gen {self.generation} connect failed on peer {self.watch.pid}: {box['err']}")
            self.aborted = True
            raise PeerFailure(f"gen {self.generation}: connect failed: {box['err']}")
        self.pg = box["pg"]
        if self.aborted:  # the watchdog aborted us while the rendezvous was finishing
            pg, self.pg = self.pg, None
            _GRAVEYARD.append(pg)
            raise PeerFailure(f"gen {self.generation}: aborted during connect")

    # ------------------------------------------------------------------ guarded wait
    def _wait(self, work, op: str):
        w = self.watch
        if w is None:
            work.wait()
            return
        if self.fault_hook is not None:
            self.fault_hook(self, op)
        if self.backend == "gloo" and op in ("send", "recv"):
            # gloo point-to-point work reports completion only from inside wait() (and a wait
            # with a timeout closes the pair), so the blocking wait runs on a helper thread that
            # is abandoned if the generation aborts
            box = {}

            def waiter():
                try:
                    work.wait()
                    box["ok"] = True
                except Exception as e:  # noqa: BLE001
                    box["err"] = e

            th = threading.Thread(target=waiter, name=f"vcx-p2p-{op}", daemon=True)
            th.start()
            while th.is_alive():
                if w.tripped():
                    self.abort()
                    raise PeerFailure(f"gen {self.generation}: {op} aborted ({w.abort_reason()})")
                th.join(self.poll_s * 5)
            if "err" in box:
                e = box["err"]
                w.declare_abort(f"{op} failed on peer {w.pid}: {type(e).__name__}: {str(e)[:120]}")
                self.abort()
                raise PeerFailure(f"gen {self.generation}: {op} failed: {e}") from e
            return
        t0 = time.perf_counter()
        while not work.is_completed():
            if w.tripped():
                self.abort()
                raise PeerFailure(f"gen {self.generation}: {op} aborted ({w.abort_reason()})")
            # spin briefly (GPU collectives finish in ~ms), then yield the GIL to the watchdog
            time.sleep(0 if time.perf_counter() - t0 < 2e-4 else self.poll_s)
        try:
            work.wait()
        except Exception as e:  # noqa: BLE001 — gloo: "Connection closed by peer", NCCL: aborted comm
            w.declare_abort(f"{op} failed on peer {w.pid}: {type(e).__name__}: {str(e)[:120]}")
            self.abort()
            raise PeerFailure(f"gen {self.generation}: {op} failed: {e}") from e

    def _check(self):
        if self._pending is not None or self._bg is not None:
            self.connect()
        if self.aborted or self.pg is None and self.size > 1:
            raise PeerFailure(f"gen {self.generation}: group aborted or never connected")
        if self.watch is not None and self.watch.tripped():
            self.abort()
            raise PeerFailure(f"gen {self.generation}: aborted ({self.watch.abort_reason()})")

    def abort(self):
        """Tear down this generation's communicator; safe to call from the watchdog thread, and
        it never blocks the caller. For RCCL, ``ncclCommAbort`` (which makes the kernels spinning
        on a dead peer exit) runs on a helper thread: it waits for RCCL's proxy thread, which
        can sit in a connect-retry loop towards a dead peer for tens of seconds, and neither the
        heartbeat thread (a silent survivor looks dead to everyone else) nor the recovering
        main thread may wait for that. The next generation uses a new communicator and new
        streams, so nothing queues behind the aborted kernels."""
        with self._abort_lock:  # exactly one caller tears the communicator down
            if self.aborted:
                return
            self.aborted = True
            pg, self.pg = self.pg, None
        if pg is None:
            return
        if self.backend == "nccl":
            th = threading.Thread(target=_abort_quietly, args=(pg,), name=f"vcx-pg{self.generation}-abort",
                                  daemon=True)
            th.start()
            _ABORTING.append((pg, th))
            return
        _abort_quietly(pg)
        _GRAVEYARD.append(pg)

    # ------------------------------------------------------------------ collectives
    def _issue(self, op: str, fn):
        """Issue one collective on this generation's communicator. The watchdog can abort the
        communicator between ``_check()`` and the issue (a member's lease expired meanwhile): the
        issue then raises (RCCL: "communicator was aborted") or finds it torn down. Under a watch that
        is the round's failure -- a PeerFailure the trainer redoes the round on -- not a crash of the
        survivor (8-rank rehearsal, round 5: survivors died of a DistBackendError raised by
        alltoall_base itself)."""
        pg = self.pg
        try:
            if pg is None:
                raise RuntimeError("communicator torn down")
            return fn(pg)
        except Exception as e:  # noqa: BLE001
            w = self.watch
            if w is None or not self._transport_failure(e):
                raise  # a caller bug (shape / split mismatch ...) stays a visible crash
            w.declare_abort(f"{op} issue failed on peer {w.pid}: {type(e).__name__}: {str(e)[:120]}")
            self.abort()
            raise PeerFailure(f"gen {self.generation}: {op} issue failed: {e}") from e

    _TRANSPORT_WORDS = ("abort", "torn down", "connection", "timed out", "timeout", "closed", "reset by peer",
                        "broken pipe", "unhandled system error", "remote process exited")

    def _transport_failure(self, e: Exception) -> bool:
        """Did the issue fail because of the communicator or a peer (-> the round's PeerFailure), rather
        than because of the call itself? Programming errors (ValueError, TypeError, IndexError, ...)
        and RuntimeErrors that name no transport condition are re-raised unchanged."""
        w = self.watch
        if self.aborted or self.pg is None or (w is not None and w.tripped()):
            return True
        for name in ("DistBackendError", "DistNetworkError", "DistStoreError"):
            cls = getattr(dist, name, None)
            if cls is not None and isinstance(e, cls):
                return True
        if isinstance(e, (ConnectionError, TimeoutError)):
            return True
        if type(e) is RuntimeError:
            msg = str(e).lower()
            return any(k in msg for k in self._TRANSPORT_WORDS)
        return False

    def allreduce_(self, t: torch.Tensor):
        if self.size == 1:
            return t
        self._check()
        self._wait(self._issue("allreduce", lambda pg: pg.allreduce([t])), "allreduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0):
        if self.size == 1:
            return t
        self._check()
        opts = dist.BroadcastOptions()
        opts.rootRank = root
        opts.rootTensor = 0
        self._wait(self._issue("broadcast", lambda pg: pg.broadcast([t], opts)), "broadcast")
        return t

    def reduce_scatter_(self, out: torch.Tensor, inp: torch.Tensor):
        """out (numel = inp.numel()/size) <- sum over peers of this peer's slice of inp."""
        if self.size == 1:
            out.copy_(inp)
            return out
        self._check()
        if self.backend == "gloo":  # gloo lacks reduce_scatter_base: all-reduce then slice
            tmp = inp.clone()
            self._wait(self._issue("reduce_scatter", lambda pg: pg.allreduce([tmp])), "reduce_scatter")
            n = out.numel()
            out.copy_(tmp[self.rank * n : (self.rank + 1) * n])
            return out
        self._wait(self._issue("reduce_scatter", lambda pg: pg._reduce_scatter_base(out, inp)), "reduce_scatter")
        return out

    def all_gather_(self, out: torch.Tensor, inp: torch.Tensor):
        if self.size == 1:
            out.copy_(inp)
            return out
        self._check()
        self._wait(self._issue("all_gather", lambda pg: pg._allgather_base(out, inp)), "all_gather")
        return out

    def all_gather_object_sizes(self, n: int):
        """All-gather one int per peer (small metadata exchange)."""
        if self.size == 1:
            return [n]
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.tensor([n], dtype=torch.int64, device=dev)
        out = torch.zeros(self.size, dtype=torch.int64, device=dev)
        self.all_gather_(out, t)
        return out.tolist()

    def send(self, t: torch.Tensor, dst: int, tag: int = 0):
        self._check()
        if self.backend == "gloo" and t.device.type != "cpu":
            t = t.to("cpu")  # gloo point-to-point moves host memory only (its collectives stage GPU tensors)
        self._wait(self._issue("send", lambda pg: pg.send([t], dst, tag)), "send")

    def recv(self, t: torch.Tensor, src: int, tag: int = 0):
        self._check()
        if self.backend == "gloo" and t.device.type != "cpu":
            host = torch.empty(t.shape, dtype=t.dtype)  # a fresh buffer: abandoned if the wait aborts
            self._wait(self._issue("recv", lambda pg: pg.recv([host], src, tag)), "recv")
            t.copy_(host)
            return
        self._wait(self._issue("recv", lambda pg: pg.recv([t], src, tag)), "recv")

    def exchange(self, send_t: torch.Tensor, recv_t: torch.Tensor, peer: int, tag: int = 0):
        """Pairwise swap with `peer`. The lower rank sends first, the higher receives first,
        which keeps blocking RCCL/gloo point-to-point deadlock-free without group calls."""
        if self.rank < peer:
            self.send(send_t, peer, tag)
            self.recv(recv_t, peer, tag)
        else:
            self.recv(recv_t, peer, tag)
            self.send(send_t, peer, tag)

    def alltoall_(self, recv_t: torch.Tensor, send_t: torch.Tensor, recv_splits, send_splits):
        """Generic variable-split all-to-all over flat buffers (RCCL: one grouped send/recv
        launch that drives every xGMI link of this GPU at once)."""
        self._check()
        self._wait(self._issue("alltoall", lambda pg: pg.alltoall_base(recv_t.view(-1), send_t.view(-1), list(recv_splits),
                                                                        list(send_splits), dist.AllToAllOptions())),
                   "alltoall")

    def exchange_all(self, send_t: torch.Tensor, recv_t: torch.Tensor, send_to: int, recv_from: int | None = None):
        """One round in which EVERY rank of the group sends `send_t` to `send_to` and receives
        `recv_t` from `recv_from` (default: the same peer). Issued as ONE alltoall whose only
        non-empty splits are those two, so RCCL runs it as grouped send/recv: both directions of
        the xGMI link at once (the blocking `exchange` above serialises them)."""
        recv_from = send_to if recv_from is None else recv_from
        ins = [0] * self.size
        outs = [0] * self.size
        ins[send_to] = send_t.numel()
        outs[recv_from] = recv_t.numel()
        self.alltoall_(recv_t, send_t, outs, ins)

    def barrier(self):
        if self.size == 1:
            return
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.zeros(1, device=dev)
        self.allreduce_(t)
        if self.backend == "nccl":
            torch.cuda.synchronize()

    def shutdown(self):
        """Release the communicator after its last use (a new generation replaces it)."""
        if self.aborted:
            return
        pg, self.pg = self.pg, None
        if pg is not None and self.backend == "nccl":
            try:
                pg.shutdown()
            except Exception:  # noqa: BLE001
                pass
