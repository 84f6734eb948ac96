"""Elastic membership for the training job: heartbeats, leases, agreed rounds, mid-collective
abort, generations, (re)join.

Reference behaviour generalised: the reference coordinator tracks its
volunteer pool through explicit ``join``/``end`` verbs only (server.py:104-154), never notices
a crashed client, and its dispatcher blocks forever in a send to a dead one (server.py:89).
Here every peer

* heartbeats a counter in the rendezvous store (``hb/<pid>``) from a background thread, which
  is also the **collective watchdog**: while this peer is inside a guarded collective it
  watches the other members' heartbeats and the generation's abort key; a member silent for
  ``lease_s`` (crashed, SIGSTOPped, partitioned) makes it post ``abort/<gen>`` and abort its
  communicator (RCCL: ``ncclCommAbort``), which unblocks the collective on every survivor;
* runs each averaging round as: arrive -> ONE agreed outcome -> guarded collectives -> ONE
  agreed verdict. The outcome of round k of generation g is a single ``compare_set`` on
  ``out/<g>/<k>`` (``same`` or ``next:<members>|<newcomers>|<joins>``) that every peer follows,
  so two peers can never disagree about whether the group changed (a joiner registering
  mid-round or a lease expiring on one peer only). The verdict (``verdict/<g>/<tag>``) is
  ``commit`` once every member reported success, or ``abort``; results are applied only on
  ``commit``, so a round that some peers finished and others did not is redone by all;
* recovers from an aborted generation with a recovery round (``out/<g>/R``): the survivors
  (members that arrive; silent ones are dropped by lease) plus pending joiners form g+1;
  the trainer restores its pre-round state and redoes the round on the new group;
* a member that arrives after it was voted out (it was stopped, or just slow) finds itself
  outside the next generation and rejoins transparently as a newcomer;
* a new or returning peer registers under ``join/<seq>`` and is admitted at the next round's
  outcome; newcomers (and any member that has not yet completed a committed round since it
  joined) receive the model inside the admission round. Staged admission (default): when the
  only change is joiners, the outcome is ``pre:<members>|<newcomers>|<joins>`` -- generation g+1
  is agreed now, the current round still runs on g, every member starts building g+1's
  communicator on a helper thread, and the group switches to g+1 at the NEXT round, whose
  admission then pays only the model broadcast (the RCCL init ran during the local steps);
* store writes and visibility: a TCPStore ``set`` is not acknowledged (the client sends it and
  returns; measured: a ``check`` on another connection right after an 8 MB ``set`` missed it 32
  times in 50), while ``add`` / ``compare_set`` / ``get`` / ``check`` are request-response and a
  connection's requests are applied in order. So every key other peers must see at a point they
  can name is posted with ``compare_set`` (abort, outcome, verdict) or followed by an ``add`` on the
  same connection (arrival); a joiner's ``join/<seq>`` record can trail its ``njoin`` ticket, and
  the scan admits joiners only up to the first ticket whose record is not visible yet
  (``_pending_joiners``) -- counting the ticket without its record lost that joiner for good;
* process death is seen at once, not after a lease: every peer listens on a TCP "liveness" port
  (published as ``live/<pid>``) and holds one connection to each other member's. Nothing is ever
  sent on them; when a peer process dies (SIGKILL, crash, OOM) its kernel closes its sockets and
  every survivor's blocking read returns EOF within milliseconds. Inside a guarded collective that
  aborts the generation right away; between rounds it marks the member dead for the next
  arrival. The lease remains the detector for what closes no socket (a hang, SIGSTOP, a
  partition).
"""
from __future__ import annotations

import os
import socket
import datetime
import threading
import time
from contextlib import contextmanager

from .. import config
from .peer_group import PeerFailure, PeerGroup

_P = "vcx/el/"


def _dbg(pid, msg):
    if config.get().elastic_debug:
        print(f"[elastic {pid} {time.time() % 1000:8.3f}] {msg}", flush=True)


def _s(v) -> str:
    return v.decode() if isinstance(v, (bytes, bytearray)) else str(v)


def _csv(xs) -> str:
    return ",".join(str(int(x)) for x in xs)


def _ints(s: str) -> list[int]:
    return [int(x) for x in s.split(",") if x]


def _parse_gen(rec: str):
    members, newcomers, njoin = rec.split("|")
    return _ints(members), _ints(newcomers), int(njoin)


def _store_host(store) -> str | None:
    """The host a (possibly prefixed) TCPStore connects to, or None for other stores."""
    seen = 0
    while store is not None and seen < 8:
        host = getattr(store, "host", None)
        if isinstance(host, str) and host:
            return host
        store = getattr(store, "underlying_store", None)
        seen += 1
    return None


def _route_ip(target: str) -> str:
    """This host's address on the route to `target` (what the other peers can connect to)."""
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect((target, 9))
            return s.getsockname()[0]
        finally:
            s.close()
    except OSError:
        return "127.0.0.1"


class _ThreadStores:
    """Per-thread clients of one store. A TCPStore client serialises its requests, so a blocking
    `wait` (a bell, a verdict) on the training thread held the heartbeat thread's `add` and the
    watchdog's abort post behind it -- up to a whole wait timeout (measured: a 0.65 s regroup round
    whose detection took 41 ms). Every other thread gets its own `clone()`."""

    def __init__(self, base):
        self.base = base
        self.owner = threading.get_ident()
        self._tls = threading.local()

    def get(self, *a):  # (named explicitly: the hottest calls skip __getattr__)
        return self.client().get(*a)

    def client(self):
        if threading.get_ident() == self.owner:
            return self.base
        c = getattr(self._tls, "c", None)
        if c is None:
            try:
                c = self.base.clone()
            except Exception:  # noqa: BLE001 — a store without clone(): share the one client
                c = self.base
            self._tls.c = c
        return c

    def __getattr__(self, name):
        return getattr(self.client(), name)


class _NoHello(ConnectionError):
    """A liveness connect reached something that is not the member's listener (no / wrong hello)."""


class _Liveness:
    """Process-death detector (see the module docstring): a listening socket whose accepted
    connections are held open (our death = their EOF) and one outgoing connection per other
    member, each read by a thread that reports EOF / error once as on_eof(member, address)."""

    def __init__(self, store, pid: int, host: str, on_eof, on_refused=None):
        self.store, self.pid, self.on_eof, self.on_refused = store, pid, on_eof, on_refused
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind(("0.0.0.0", 0))
        self.srv.listen(128)
        self.addr = f"{host}:{self.srv.getsockname()[1]}"
        self._held: list[socket.socket] = []
        self._conn: dict[int, tuple[str, socket.socket]] = {}
        # member -> (address, time) of a connect attempt in flight or one that failed recently: a
        # failed connect proves nothing (wrong route, firewall, a peer still starting), so it is
        # retried after retry_s and never reported as death -- the lease covers that member
        self._trying: dict[int, tuple[str, float]] = {}
        self.retry_s = 2.0
        self.connect_failures = 0
        self._lock = threading.Lock()
        self._stop = threading.Event()
        threading.Thread(target=self._accept, name=f"vcx-live-acc-{pid}", daemon=True).start()
        store.set(f"{_P}live/{pid}", self.addr)

    def _accept(self):
        while not self._stop.is_set():
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            try:  # the hello that makes the connector's link count as established (see _connect)
                c.sendall(self._hello(self.pid))
            except OSError:
                c.close()
                continue
            with self._lock:
                self._held.append(c)

    @staticmethod
    def _hello(pid: int) -> bytes:
        return f"vcxlive {pid}\n".encode()

    def address_of(self, m: int) -> str | None:
        key = f"{_P}live/{m}"
        try:
            return _s(self.store.get(key)) if self.store.check([key]) else None
        except Exception:  # noqa: BLE001
            return None

    def watch(self, members):
        """Hold a connection to every member (new ones, or a restarted one's new address). Connects
        run on their own threads, so an unreachable address never stalls the caller (the heartbeat
        thread); only an EOF on an ESTABLISHED connection reports a death."""
        now = time.time()
        for m in members:
            if m == self.pid or self._stop.is_set():
                continue
            addr = self.address_of(m)
            with self._lock:
                cur = self._conn.get(m)
                tr = self._trying.get(m)
                if addr is None or (cur is not None and cur[0] == addr):
                    continue
                if tr is not None and tr[0] == addr and (tr[1] < 0 or now - tr[1] < self.retry_s):
                    continue  # a connect in flight (time < 0), or it failed a moment ago
                self._trying[m] = (addr, -1.0)
            threading.Thread(target=self._connect, args=(m, addr), name=f"vcx-live-con-{self.pid}-{m}",
                             daemon=True).start()

    def _connect(self, m, addr):
        host, _, port = addr.rpartition(":")
        try:
            c = socket.create_connection((host, int(port)), timeout=2.0)
            try:
                # established = member m's listener answered with its hello: a middlebox that accepts
                # and closes (or a stranger now on that port) is a failed connect, never a death
                want, buf = self._hello(m), b""
                while len(buf) < len(want):
                    part = c.recv(len(want) - len(buf))
                    if not part:
                        raise _NoHello(f"closed before the liveness hello ({buf!r})")
                    buf += part
                if buf != want:
                    raise _NoHello(f"unexpected liveness hello {buf!r}")
                c.settimeout(None)
            except OSError:
                c.close()
                raise
        except OSError as e:
            with self._lock:
                self.connect_failures += 1
                if self._trying.get(m, (None,))[0] == addr:
                    self._trying[m] = (addr, time.time())  # retried after retry_s; not a death
            _dbg(self.pid, f"liveness connect to peer {m} at {addr} failed ({e!r}); lease-only until it succeeds")
            # refused, or accepted and then closed / reset without the hello (the member died between
            # its kernel's accept and its listener's hello -- or a middlebox): a hint only, the
            # membership declares the death only if the member's heartbeat also stands still
            if isinstance(e, (ConnectionRefusedError, ConnectionResetError, _NoHello)) and self.on_refused is not None:
                self.on_refused(m, addr)
            return
        with self._lock:
            if self._stop.is_set():
                c.close()
                return
            old = self._conn.get(m)
            self._conn[m] = (addr, c)
            self._trying.pop(m, None)
        if old is not None:
            try:
                old[1].close()
            except OSError:
                pass
        threading.Thread(target=self._read, args=(m, addr, c), name=f"vcx-live-{self.pid}-{m}",
                         daemon=True).start()

    def _read(self, m, addr, c):
        try:
            while c.recv(64):
                pass
        except OSError:
            pass
        with self._lock:
            mine = self._conn.get(m, (None, None))[1] is c
        if mine and not self._stop.is_set():
            self.on_eof(m, addr)

    def close(self):
        self._stop.set()
        with self._lock:
            socks = [c for _, c in self._conn.values()] + self._held
            self._conn.clear()
            self._held.clear()
        for c in socks + [self.srv]:
            try:
                c.close()
            except OSError:
                pass


class ElasticMembership:
    def __init__(self, store, peer_id: int, *, backend: str = "gloo", device=None, lease_s: float = 3.0,
                 heartbeat_s: float = 0.2, arrive_timeout_s: float = 600.0, pg_timeout_s: float | None = None,
                 poll_s: float = 0.002, liveness: bool | None = None, live_host: str | None = None):
        self._stores = store if isinstance(store, _ThreadStores) else _ThreadStores(store)
        self.pid = int(peer_id)
        self.backend = backend
        self.device = device
        self.lease_s = lease_s
        self.heartbeat_s = heartbeat_s
        self.arrive_timeout_s = arrive_timeout_s
        # a gloo op blocked on a stopped peer is only freed by this timeout (gloo cannot cancel)
        self.pg_timeout_s = pg_timeout_s if pg_timeout_s is not None else max(60.0, 30.0 * lease_s)
        self.poll_s = poll_s
        self.gen = -1
        self.members: list[int] = []
        self.prev_members: list[int] = []
        self.newcomers: list[int] = []
        self.group: PeerGroup | None = None
        self.round = 0
        self.joins_seen = 0
        self._join_gap: dict[int, float] = {}  # join ticket -> when its record was first found missing
        self.has_model = True
        self.fault_hook = None  # passed to every generation's PeerGroup (fault-injection tests)
        self.failures = 0
        self.events: list[dict] = []  # membership change log (for metrics / tests)
        self._hb_stop = threading.Event()
        self._wake = threading.Event()
        self._hb_thread = None
        self._lock = threading.RLock()
        self._armed = False
        self._abort = threading.Event()
        self._abort_reason = ""
        self._watch_seen: dict[int, tuple[int, float]] = {}
        # liveness links: member -> the address of the incarnation whose connection hit EOF
        self.liveness = config.get().elastic_liveness if liveness is None else liveness
        # published liveness address: this host's address on the route to the rendezvous store
        # (the one host every member reaches), not MASTER_ADDR, which a --coordinator run never sets
        self.live_host = live_host or _route_ip(_store_host(self._stores.base)
                                                or os.environ.get("MASTER_ADDR", "127.0.0.1"))
        self._live: _Liveness | None = None
        self._eof: dict[int, str] = {}
        # member -> (address, heartbeat count, time of the first refusal, refusals) of refused liveness
        # connects: a refusal is only a hint (NAT, overlapping container addresses), so the member is
        # dead only after refuse_min consecutive refusals of the same address with its heartbeat
        # standing still for refuse_grace_s since the first one (one refusal plus a 0.6 s
        # GIL / store stall of its heartbeat evicted live peers). Connects are retried every 2 s, so
        # a death found this way takes >= 2 s; a peer that dies AFTER we connected is an EOF instead.
        self._refused: dict[int, tuple[str, int, float, int]] = {}
        self.refuse_min = 2
        self.refuse_grace_s = max(2.0, 3.0 * heartbeat_s)
        self.eof_events: list[tuple[int, float]] = []  # (member, time) of every EOF seen
        self._ring_pending = False  # an EOF arrived: the heartbeat thread rings the round's bell
        self._tag = ""  # the armed guard's round tag (its verdict key is posted on a trip)
        self._gc: dict[tuple[int, int], list[str]] = {}  # (gen, round) -> keys to delete later
        # blocking store waits (server-side wake-up) instead of sleep-polling on the fast paths; a
        # wait that runs out falls back to the polling scan, which owns lease/EOF detection
        self.bell_s = min(2.0, max(0.25, lease_s / 4))
        # staged admission (the next generation's communicator built in the background during the local
        # steps) runs on gloo groups only. On RCCL it was removed in round 5: building the new
        # communicator on a helper thread while the main thread ran collectives on the current one
        # SIGSEGVed every member at 8 ranks (gpurun_out/f2/rejoin_n8_staged.log, round 4), and its
        # members' stall is accounted instead (LocalSGDTrainer.last_round_stages: the new group's
        # communicator init is its first collective, timed apart from the model broadcast)
        self.stage_joins = config.get().elastic_stage_joins == "gloo" and backend == "gloo"
        self.last_go_wait_ms = 0.0
        self._staged = None  # (gen, members, newcomers, njoin, group) agreed, built in the background
        self._retired: list = []  # groups replaced by a staged generation, shut down after its first commit
        if backend == "nccl":
            # abortable (non-blocking) RCCL communicator init for every generation's group
            os.environ.setdefault("TORCH_NCCL_USE_COMM_NONBLOCKING", "1")
            # a collective that outlives the group timeout (e.g. its abort is slow) must not take
            # the survivor down: c10d's watchdog then only aborts the communicator (CleanUpOnly)
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")

    @property
    def store(self):
        """This thread's client of the rendezvous store (see _ThreadStores)."""
        return self._stores.client()

    # ------------------------------------------------------------------ heartbeat + watchdog
    def start_heartbeat(self):
        if self._hb_thread is not None:
            return
        self._hb_stop.clear()

        def loop():
            key = f"{_P}hb/{self.pid}"
            while True:
                # a liveness EOF wakes this thread at once (the watchdog acts on it here, on the
                # one thread that has always owned aborts), otherwise one tick per heartbeat_s
                self._wake.wait(self.heartbeat_s)
                self._wake.clear()
                if self._hb_stop.is_set():
                    break
                try:
                    self.store.add(key, 1)
                except Exception:  # noqa: BLE001 — the store is gone: nothing left to do
                    return
                live = self._live
                if live is not None:
                    try:
                        live.watch(list(self.members))
                    except Exception:  # noqa: BLE001 — best effort; the lease still applies
                        pass
                if self._ring_pending:
                    # wake the peers blocked on this round's bell: their scan sees the EOF now
                    self._ring_pending = False
                    try:
                        self.store.set(f"{_P}bell/{self.gen}/{self.round}", "eof")
                    except Exception:  # noqa: BLE001
                        pass
                if self._armed:
                    try:
                        self._watch()
                    except Exception as e:  # noqa: BLE001
                        self._trip(f"watchdog error: {e!r}")

        self.store.add(f"{_P}hb/{self.pid}", 1)
        if self.liveness and self._live is None:
            self._live = _Liveness(self._stores, self.pid, self.live_host, self._on_eof, self._on_refused)
        self._hb_thread = threading.Thread(target=loop, name=f"vcx-hb-{self.pid}", daemon=True)
        self._hb_thread.start()

    def stop_heartbeat(self):
        self._hb_stop.set()
        self._wake.set()
        if self._hb_thread is not None:
            self._hb_thread.join(timeout=2)
        self._hb_thread = None
        if self._live is not None:
            self._live.close()
            self._live = None

    def _on_eof(self, m: int, addr: str):
        """A member's liveness connection closed: that process is gone."""
        now = time.time()
        with self._lock:
            self._eof[m] = addr
            self.eof_events.append((m, now))
            self._ring_pending = True
        _dbg(self.pid, f"liveness EOF from peer {m} ({addr})")
        self._wake.set()  # the watchdog (heartbeat thread) aborts a collective in flight right away

    def _on_refused(self, m: int, addr: str):
        try:
            hb = self._hb(m)
        except Exception:  # noqa: BLE001
            return
        with self._lock:
            r = self._refused.get(m)
            if r is not None and r[0] == addr and r[1] == hb:
                self._refused[m] = (addr, hb, r[2], r[3] + 1)  # the same standing incarnation again
            else:
                self._refused[m] = (addr, hb, time.time(), 1)

    def _dead(self, m: int) -> bool:
        """Member m's process is known to be gone: its established liveness link hit EOF, or its
        published address refused refuse_min connects in a row while its heartbeat stood still for
        refuse_grace_s."""
        if m in self._eof and self._gone(m):
            return True
        with self._lock:
            r = self._refused.get(m)
        if r is None or self._live is None:
            return False
        addr, hb0, t0, n = r
        if self._live.address_of(m) != addr or self._hb(m) != hb0:
            with self._lock:
                if self._refused.get(m) == r:
                    del self._refused[m]  # restarted, or alive behind a route we cannot use
            return False
        return n >= self.refuse_min and time.time() - t0 > self.refuse_grace_s

    def _gone(self, m: int) -> bool:
        """Did the connection to member m's CURRENT incarnation close (a restarted peer publishes
        a new address and is not 'gone')?"""
        with self._lock:
            addr = self._eof.get(m)
        if addr is None or self._live is None:
            return False
        return self._live.address_of(m) == addr

    def _watch(self):
        """One watchdog tick while a guarded collective is in flight."""
        if self._abort.is_set():
            return
        g = self.gen
        ak = f"{_P}abort/{g}"
        if self.store.check([ak]):
            self._trip(_s(self.store.get(ak)))
            return
        now = time.time()
        for m in list(self.members):
            if m == self.pid:
                continue
            if self._dead(m):  # its liveness link closed (or refused, heartbeat still): the process is gone
                self.declare_abort(f"peer {m} process gone (liveness EOF) during a collective of gen {g}")
                return
            hb = self._hb(m)
            last = self._watch_seen.get(m)
            if last is None or hb != last[0]:
                self._watch_seen[m] = (hb, now)
            elif now - last[1] > self.lease_s:
                self.declare_abort(f"peer {m} silent for {now - last[1]:.2f}s inside a collective of gen {g}")
                return

    def declare_abort(self, reason: str):
        """Abort the current generation for everyone: post the abort key, trip locally."""
        try:
            self.store.compare_set(f"{_P}abort/{self.gen}", "", reason)
        except Exception:  # noqa: BLE001
            pass
        self._trip(reason)

    def _trip(self, reason: str):
        with self._lock:
            if self._abort.is_set():
                return
            self._abort_reason = reason
            self._abort.set()
            grp = self.group
            tag = self._tag if self._armed else ""
        if tag:  # peers blocked on this round's verdict wake up to the abort
            self._vote(tag, "abort")
        self.events.append({"event": "abort", "gen": self.gen, "reason": reason, "t": time.time()})
        _dbg(self.pid, f"trip gen {self.gen}: {reason}")
        if grp is not None:
            grp.abort()  # RCCL: ncclCommAbort — kernels blocked on the dead peer exit

    def tripped(self) -> bool:
        return self._abort.is_set()

    def abort_reason(self) -> str:
        return self._abort_reason

    # ------------------------------------------------------------------ bootstrap / join / leave
    def bootstrap(self, members: list[int]):
        """Generation 0 with a known member list (e.g. all torchrun ranks)."""
        members = sorted(int(m) for m in members)
        rec = _s(self.store.compare_set(f"{_P}gen/0", "", f"{_csv(members)}||0"))
        m0, nc0, nj0 = _parse_gen(rec)
        self._adopt(0, m0, nc0, nj0)
        self.start_heartbeat()
        return self.group

    def join(self, timeout_s: float = 600.0):
        """Ask to be admitted; blocks until a generation that contains this peer forms."""
        self.start_heartbeat()
        try:
            self.store.delete_key(f"{_P}leave/{self.pid}")
        except Exception:  # noqa: BLE001
            pass
        self.has_model = False
        seq = int(self.store.add(f"{_P}njoin", 1))
        self.store.set(f"{_P}join/{seq}", str(self.pid))
        g = self._latest_gen(max(self.gen, 0))
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            key = f"{_P}gen/{g + 1}"
            if self.store.check([key]):
                members, newcomers, njoin = _parse_gen(_s(self.store.get(key)))
                if self.pid in members and njoin >= seq:
                    self._adopt(g + 1, members, newcomers, njoin)
                    self.group.needs_go = True  # line up with the continuing members (guard)
                    self.events.append({"event": "joined", "gen": self.gen, "members": members})
                    return self.group
                if njoin >= seq:
                    # our ticket was counted without us (its record reached the store after the
                    # members gave up waiting for it, see _pending_joiners): take a new one
                    seq = int(self.store.add(f"{_P}njoin", 1))
                    self.store.set(f"{_P}join/{seq}", str(self.pid))
                g += 1
                continue
            time.sleep(0.01)
        raise TimeoutError(f"peer {self.pid}: not admitted within {timeout_s}s")

    def leave(self):
        """Graceful leave: survivors drop this peer at their next round without a lease wait."""
        self.store.set(f"{_P}leave/{self.pid}", str(self.gen))
        self.stop_heartbeat()
        self._drop_group()
        self._drop_staged()
        self._release_retired()

    # ------------------------------------------------------------------ rounds
    def sync_round(self):
        """Start the next averaging round of the current generation. Returns
        (group, changed, newcomers); if this peer was voted out it rejoins transparently."""
        if self._abort.is_set() or self.store.check([f"{_P}abort/{self.gen}"]):
            return self.recover()
        if self._staged is not None:
            return self._switch()
        self.round += 1
        self._collect(self.round - 2)
        return self._round(str(self.round), recovery=False)

    def _collect(self, r: int):
        """Delete round r's keys of the current generation: every member has passed round r+1
        (its guard could not commit otherwise), so nothing reads them again."""
        keys = self._gc.pop((self.gen, r), None)
        for key in keys or ():
            try:
                self.store.delete_key(key)
            except Exception:  # noqa: BLE001
                pass
        for stale in [gk for gk in self._gc if gk[0] != self.gen]:
            self._gc.pop(stale)  # an old generation's keys stay (an evicted peer may still read them)

    def _mark(self, r, *keys):
        self._gc.setdefault((self.gen, r), []).extend(keys)

    def recover(self):
        """After a PeerFailure: leave the aborted generation and form the next one from the
        members that arrive (silent ones are dropped by lease) plus pending joiners."""
        g = self.gen
        self.failures += 1
        try:
            self.store.compare_set(f"{_P}abort/{g}", "", f"recovery requested by peer {self.pid}")
        except Exception:  # noqa: BLE001
            pass
        self._trip(f"recovery of gen {g}")
        return self._round("R", recovery=True)

    @contextmanager
    def guard(self, phase: str = ""):
        """Arm the watchdog around the collectives of one round, then agree on the verdict.
        Raises PeerFailure (after voting abort) if any member failed; the caller restores its
        pre-round state and calls ``recover()``. Nothing may be applied before this exits."""
        grp = self.group
        if grp is None or grp.size == 1:
            yield
            if grp is not None:
                self.has_model = True
            return
        tag = f"{self.round}{phase}"
        with self._lock:
            if self._abort.is_set():
                raise PeerFailure(f"gen {self.gen}: aborted ({self._abort_reason})")
            self._watch_seen = {}
            self._tag = tag
            if self.pid == self.members[0]:
                self._mark(self.round, f"{_P}ok/{self.gen}/{tag}", f"{_P}verdict/{self.gen}/{tag}")
            self._armed = True
        try:
            _dbg(self.pid, f"guard {self.gen}/{tag}: connect")
            fresh = not getattr(grp, "_connected", True) or getattr(grp, "_pending", None) is not None
            t0 = time.time()
            grp.connect()
            if fresh:  # communicator build of a new generation (RCCL init / gloo full mesh)
                self.events.append({"event": "connect", "gen": self.gen, "ms": (time.time() - t0) * 1e3,
                                    "t": time.time(), "bg_build_ms": getattr(grp, "bg_build_ms", None)})
            if getattr(grp, "needs_go", False):
                self.wait_round_start()
                grp.needs_go = False
                self.events.append({"event": "go", "gen": self.gen, "ms": self.last_go_wait_ms, "t": time.time()})
            _dbg(self.pid, f"guard {self.gen}/{tag}: body")
            yield
            _dbg(self.pid, f"guard {self.gen}/{tag}: commit")
            self._commit(tag)
            self._release_retired()
            st = self._staged
            if st is not None and not st[4]._connected and st[4]._bg is None:
                st[4].start_connect()  # the staged generation builds during the local steps
        except PeerFailure:
            self._vote(tag, "abort")
            raise
        finally:
            self._armed = False

    def _vote(self, tag, v):
        try:
            return _s(self.store.compare_set(f"{_P}verdict/{self.gen}/{tag}", "", v))
        except Exception:  # noqa: BLE001
            return "abort"

    def _wait_keys(self, keys, timeout_s: float) -> bool:
        """Block until every key exists (the store wakes us), or the timeout passes."""
        try:
            self.store.wait(keys, datetime.timedelta(seconds=timeout_s))
            return True
        except Exception:  # noqa: BLE001 — DistStoreError on timeout
            return False

    def _commit(self, tag):
        g, P = self.gen, len(self.members)
        okk, vk = f"{_P}ok/{g}/{tag}", f"{_P}verdict/{g}/{tag}"
        if int(self.store.add(okk, 1)) >= P:
            v = self._vote(tag, "commit")  # the last member in: everyone's body completed
        else:
            # everyone else blocks on the verdict key: written by the last member in, by a member
            # whose body failed, or by a watchdog trip (EOF / lease) of any member
            while True:
                if self._wait_keys([vk], self.bell_s):
                    v = _s(self.store.get(vk))
                    break
                if self._abort.is_set():
                    v = self._vote(tag, "abort")
                    break
                if int(self.store.add(okk, 0)) >= P:
                    v = self._vote(tag, "commit")
                    break
        _dbg(self.pid, f"verdict {g}/{tag}: {v}")
        if v != "commit":
            self._trip(f"round {g}/{tag} voted abort")
            raise PeerFailure(f"gen {g}: round {tag} aborted ({self._abort_reason})")
        self.has_model = True

    def _round(self, k: str, recovery: bool):
        g = self.gen
        # stall anatomy of a round that ends in a new generation (reported on its regroup event)
        self._rt = {"t_in": time.time(), "bell_wait_ms": 0.0, "scan_ms": 0.0}
        self.store.set(f"{_P}arr/{g}/{k}/{self.pid}", "1" if self.has_model else "0")
        okey = f"{_P}out/{g}/{k}"
        bell = f"{_P}bell/{g}/{k}"
        if not recovery:
            self._mark(self.round, f"{_P}arr/{g}/{k}/{self.pid}")
            if self.members and self.pid == self.members[0]:
                self._mark(self.round, f"{_P}narr/{g}/{k}", okey, bell)
            # fast path (every member arrives, nobody joins): the last one in proposes "same" and
            # rings the bell; the others sleep in a store wait instead of scanning the members
            n = int(self.store.add(f"{_P}narr/{g}/{k}", 1))
            if n >= len(self.members):
                if self._njoin() <= self.joins_seen:
                    self.store.compare_set(okey, "", "same")
                    self.store.set(bell, "1")
                    return self._follow(okey)
            elif not any(m != self.pid and self._dead(m) for m in self.members):
                # (a member whose link already closed will not arrive: straight to the scan)
                tw = time.time()
                rang = self._wait_keys([bell], self.bell_s)
                self._rt["bell_wait_ms"] = (time.time() - tw) * 1e3
                if rang and self.store.check([okey]):
                    return self._follow(okey)
        others = [m for m in self.members if m != self.pid]
        now = time.time()
        t_scan = now
        hb_seen = {}
        for m in others:
            # recovery: a member the watchdog already saw silent keeps its silence clock (the
            # aborted round's lease wait is not paid a second time before it is declared dead)
            hb = self._hb(m)
            ws = self._watch_seen.get(m) if recovery else None
            hb_seen[m] = (hb, ws[1]) if ws is not None and ws[0] == hb else (hb, now)
        arrived = {self.pid: self.has_model}
        dead, left = set(), set()
        t0 = now
        nj_cached, joiners, njoin = -1, [], self.joins_seen
        while True:
            if self.store.check([okey]):
                return self._follow(okey)
            if not recovery and self.store.check([f"{_P}abort/{g}"]):
                return self.recover()
            nj_raw = self._njoin()
            if nj_raw != nj_cached or njoin < nj_raw:  # new tickets, or records still on their way
                (joiners, njoin), nj_cached = self._pending_joiners(nj_raw), nj_raw
            missing = []
            for m in others:
                if m in arrived or m in dead or m in left:
                    continue
                ak = f"{_P}arr/{g}/{k}/{m}"
                if self.store.check([ak]):
                    arrived[m] = _s(self.store.get(ak)) == "1"
                    continue
                if m in joiners or self.store.check([f"{_P}leave/{m}"]):
                    left.add(m)  # announced leave, or restarted and re-registered as a joiner
                    continue
                if self._dead(m):
                    dead.add(m)  # its liveness link closed: no lease wait
                    continue
                hb = self._hb(m)
                last, seen_at = hb_seen[m]
                if hb != last:
                    hb_seen[m] = (hb, time.time())
                elif time.time() - seen_at > self.lease_s:
                    dead.add(m)
                    continue
                missing.append(m)
            if not missing:
                break
            if time.time() - t0 > self.arrive_timeout_s:
                dead.update(missing)
                break
            time.sleep(self.poll_s)
        if not recovery and not dead and not left and njoin <= self.joins_seen:
            decision = "same"
        else:
            survivors = sorted(arrived)
            new_ids = [j for j in joiners if j not in arrived]
            members = sorted(set(survivors) | set(new_ids))
            newcomers = sorted(set([m for m in survivors if not arrived[m]] + new_ids))
            # only joiners, every member holds the model: stage the generation (see module docstring)
            kind = "pre" if (self.stage_joins and not recovery and not dead and not left and new_ids
                             and all(arrived.values())) else "next"
            decision = f"{kind}:{_csv(members)}|{_csv(newcomers)}|{njoin}"
        self._rt["scan_ms"] = (time.time() - t_scan) * 1e3
        won = _s(self.store.compare_set(okey, "", decision))
        self.store.set(bell, "1")
        _dbg(self.pid, f"round {g}/{k}: proposed {decision!r} (dead={sorted(dead)} left={sorted(left)}), agreed {won!r}")
        return self._follow(okey)

    # ------------------------------------------------------------------ internals
    def _follow(self, okey):
        v = _s(self.store.get(okey))
        if v == "same":
            return self.group, False, []
        g = self.gen + 1
        kind, body = v.split(":", 1)
        # every follower proposes the same record; the first write fixes generation g
        rec = _s(self.store.compare_set(f"{_P}gen/{g}", "", body))
        members, newcomers, njoin = _parse_gen(rec)
        if kind == "pre" and rec == body and self.pid in members:
            self._stage(g, members, newcomers, njoin)
            return self.group, False, []  # this round still runs on the current generation
        old = list(self.members)
        k = okey.rsplit("/", 1)[1]
        if self.pid not in members:
            # voted out (stopped, partitioned or late): rejoin as a newcomer
            self.events.append({"event": "evicted", "gen": g, "round": k})
            self._drop_group()
            self.gen = g
            self.join()
            return self.group, True, list(self.newcomers)
        t_dec = time.time()
        self._adopt(g, members, newcomers, njoin)
        rt = getattr(self, "_rt", None) or {}
        t = time.time()
        self.events.append({"event": "regroup", "gen": g, "members": members, "round": k,
                            "dropped": sorted(set(old) - set(members)), "joined": newcomers,
                            "t": t, "t_in": rt.get("t_in"), "bell_wait_ms": rt.get("bell_wait_ms"),
                            "scan_ms": rt.get("scan_ms"),
                            "decide_ms": (t_dec - rt["t_in"]) * 1e3 if rt.get("t_in") else None,
                            "adopt_ms": (t - t_dec) * 1e3})
        return self.group, True, newcomers

    def _stage(self, g, members, newcomers, njoin):
        """Generation g (the current members + joiners) is agreed: its group (on a store client of its
        own) starts building after this round's collectives commit; ``sync_round`` switches to it
        next round."""
        try:
            st = self._stores.base.clone()
        except Exception:  # noqa: BLE001
            st = self.store
        grp = PeerGroup(st, members.index(self.pid), len(members), self.backend, generation=g, members=members,
                        timeout_s=self.pg_timeout_s, device=self.device, watch=self)
        grp.fault_hook = self.fault_hook
        grp.needs_go = True  # its first collective is not lined up by a communicator init (guard)
        # its build starts once this round's collectives have committed (guard): an RCCL init running
        # beside another communicator's collectives broke them at 8 ranks (connects refused), and
        # between the commit and the switch there are only the local steps
        self._staged = (g, list(members), list(newcomers), int(njoin), grp)
        self.joins_seen = max(self.joins_seen, int(njoin))
        self.events.append({"event": "staged", "gen": g, "members": list(members), "joined": list(newcomers),
                            "t": time.time()})
        if self._live is not None:
            self._live.watch(members)  # liveness links to the joiners before their admission round
        _dbg(self.pid, f"staged gen {g}: {members} (+{newcomers})")

    def _switch(self):
        """Move to the staged generation (its communicator has been building since the last round)."""
        g, members, newcomers, njoin, _ = self._staged
        old = list(self.members)
        t_in = time.time()
        self._adopt(g, members, newcomers, njoin)
        t = time.time()
        self.events.append({"event": "regroup", "gen": g, "members": members, "round": "staged",
                            "dropped": sorted(set(old) - set(members)), "joined": newcomers, "t": t, "t_in": t_in,
                            "bell_wait_ms": 0.0, "scan_ms": 0.0, "decide_ms": 0.0, "adopt_ms": (t - t_in) * 1e3})
        return self.group, True, list(newcomers)

    def _drop_staged(self):
        st, self._staged = self._staged, None
        if st is not None:
            st[4].abort()

    def wait_round_start(self, timeout_s: float | None = None):
        """Inside the admission guard: block until EVERY continuing member has entered this
        generation (each adds 1 to ``go/<gen>`` when it adopts it). A staged generation's
        communicator was built rounds ago, so nothing else lines its members up before the first
        collective -- and RCCL opens that collective's connections lazily: a peer that enters it
        while another is still in its local steps has its connects refused until it gives up
        (seen at 8 ranks). Aborts like a collective if a member dies meanwhile. Records the wait
        in ``last_go_wait_ms``."""
        n_cont = sum(1 for m in self.members if m not in self.newcomers)
        t0 = time.time()
        self.last_go_wait_ms = 0.0
        if n_cont == 0:
            return  # nobody holds a model: no admission transfer to line up
        key = f"{_P}go/{self.gen}"
        while int(self.store.add(key, 0)) < n_cont:
            if self._abort.is_set():
                raise PeerFailure(f"gen {self.gen}: aborted before the admission round ({self._abort_reason})")
            if timeout_s is not None and time.time() - t0 > timeout_s:
                raise PeerFailure(f"gen {self.gen}: the members did not all enter the admission round in {timeout_s}s")
            time.sleep(self.poll_s)
        self.last_go_wait_ms = (time.time() - t0) * 1e3

    def _drop_group(self, defer: bool = False):
        with self._lock:
            grp, self.group = self.group, None
            self._armed = False
        if grp is None:
            return
        if defer:
            # switching to a staged generation whose RCCL init may still be running: destroying
            # the old communicator now blocked inside ncclCommDestroy at 8 ranks (stacks in
            # gpurun_out/i/rejoin_n8_staged.log); it is released after the next committed round
            self._retired.append(grp)
        else:
            grp.shutdown()

    def _release_retired(self):
        while self._retired:
            self._retired.pop().shutdown()

    def _adopt(self, g, members, newcomers, njoin):
        self._drop_group(defer=self._staged is not None and self._staged[0] == g)
        with self._lock:
            self._abort.clear()
            self._abort_reason = ""
        self.prev_members = list(self.members) if self.gen >= 0 else list(members)
        self.gen = g
        self.members = list(members)
        self.newcomers = list(newcomers)
        self.round = 0
        self.joins_seen = max(self.joins_seen, int(njoin))
        if self.pid in newcomers:
            self.has_model = False
        staged, self._staged = self._staged, None
        if staged is not None and staged[0] == g and staged[1] == list(members):
            grp = staged[4]  # its communicator is already building (or built)
        else:
            if staged is not None:
                staged[4].abort()  # superseded (a recovery formed another generation)
            grp = PeerGroup(self.store, members.index(self.pid), len(members), self.backend, generation=g,
                            members=members, timeout_s=self.pg_timeout_s, device=self.device, watch=self)
            grp.fault_hook = self.fault_hook
        with self._lock:
            self.group = grp
        if self._live is not None:
            self._live.watch(members)
        if self.has_model:
            try:  # counted by wait_round_start
                self.store.add(f"{_P}go/{g}", 1)
            except Exception:  # noqa: BLE001
                pass

    def _hb(self, m) -> int:
        return int(self.store.add(f"{_P}hb/{m}", 0))

    def _njoin(self) -> int:
        return int(self.store.add(f"{_P}njoin", 0))

    def _pending_joiners(self, njoin):
        """(joiners, upto): the peers behind join tickets joins_seen+1 .. upto, where upto stops in
        front of the first ticket whose ``join/<seq>`` record is not visible yet (the joiner takes
        its ticket with an acknowledged ``add`` and then posts the record with an unacknowledged
        ``set``). A ticket whose record stays missing for lease_s (the joiner died between the two)
        is skipped, so it cannot hold back the joiners behind it."""
        out = []
        upto = self.joins_seen
        now = time.time()
        for seq in range(self.joins_seen + 1, njoin + 1):
            key = f"{_P}join/{seq}"
            if self.store.check([key]):
                pid = int(_s(self.store.get(key)))
                if pid not in out:
                    out.append(pid)
            else:
                t0 = self._join_gap.setdefault(seq, now)
                if now - t0 <= self.lease_s:
                    break
            upto = seq
        return out, upto

    def _latest_gen(self, start: int = 0) -> int:
        g = start
        while self.store.check([f"{_P}gen/{g + 1}"]):
            g += 1
        return g
