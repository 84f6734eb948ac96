"""Elastic membership for the training job: heartbeats, leases, generations, (re)join.

Reference behaviour generalised: the reference coordinator tracks
its volunteer pool through explicit ``join``/``end`` verbs only (server.py:104-154) and never
notices a crashed client. Here every peer

* heartbeats a counter in the rendezvous store (``hb/<pid>``) from a background thread;
* at each averaging round posts an arrival key and waits for the other members;
* a member that has not arrived and whose heartbeat counter has not moved for ``lease_s``
  seconds is declared dead; a member that announced ``leave`` is dropped immediately;
* the survivors agree on the next generation's member list through ONE ``compare_set``
  (first proposal wins, everyone adopts it), then build a fresh ``PeerGroup`` for it —
  no collective is ever issued to a dead peer, so RCCL never hangs on one;
* a new or returning peer registers under ``join/<seq>`` and is admitted at the next round;
  the new generation's rank 0 then broadcasts the averaged model to it.
"""
from __future__ import annotations

import threading
import time

from .peer_group import PeerGroup

_P = "vcx/el/"


def _s(v) -> str:
    return v.decode() if isinstance(v, (bytes, bytearray)) else str(v)


class ElasticMembership:
    def __init__(self, store, peer_id: int, *, backend: str = "gloo", device=None, lease_s: float = 3.0,
                 heartbeat_s: float = 0.2, arrive_timeout_s: float = 600.0, pg_timeout_s: float = 300.0,
                 poll_s: float = 0.002):
        self.store = store
        self.pid = int(peer_id)
        self.backend = backend
        self.device = device
        self.lease_s = lease_s
        self.heartbeat_s = heartbeat_s
        self.arrive_timeout_s = arrive_timeout_s
        self.pg_timeout_s = pg_timeout_s
        self.poll_s = poll_s
        self.gen = -1
        self.members: list[int] = []
        self.prev_members: list[int] = []
        self.newcomers: list[int] = []
        self.group: PeerGroup | None = None
        self.round = 0
        self.joins_seen = 0
        self._hb_stop = threading.Event()
        self._hb_thread = None
        self.events: list[dict] = []  # membership change log (for metrics / tests)

    # ------------------------------------------------------------------ heartbeat
    def start_heartbeat(self):
        if self._hb_thread is not None:
            return

        def loop():
            key = f"{_P}hb/{self.pid}"
            while not self._hb_stop.wait(self.heartbeat_s):
                try:
                    self.store.add(key, 1)
                except Exception:
                    return

        self.store.add(f"{_P}hb/{self.pid}", 1)
        self._hb_thread = threading.Thread(target=loop, name=f"vcx-hb-{self.pid}", daemon=True)
        self._hb_thread.start()

    def stop_heartbeat(self):
        self._hb_stop.set()
        if self._hb_thread is not None:
            self._hb_thread.join(timeout=2)
        self._hb_thread = None

    # ------------------------------------------------------------------ bootstrap
    def bootstrap(self, members: list[int]):
        """Generation 0 with a known member list (e.g. all torchrun ranks)."""
        members = sorted(int(m) for m in members)
        self.store.compare_set(f"{_P}gen/0/members", "", ",".join(map(str, members)))
        self.store.compare_set(f"{_P}gen/0/joins", "", "0")
        self._adopt(0, members)
        self.start_heartbeat()
        return self.group

    def join(self, timeout_s: float = 600.0):
        """Ask to be admitted; blocks until a generation that contains this peer forms."""
        self.start_heartbeat()
        seq = self.store.add(f"{_P}njoin", 1)
        self.store.set(f"{_P}join/{seq}", str(self.pid))
        t0 = time.time()
        g = max(self._latest_gen(), 0)
        while time.time() - t0 < timeout_s:
            key = f"{_P}gen/{g + 1}/members"
            if self.store.check([key]):
                members = [int(x) for x in _s(self.store.get(key)).split(",") if x]
                if self.pid in members:
                    self._adopt(g + 1, members)
                    self.events.append({"event": "joined", "gen": self.gen, "members": members})
                    return self.group
                g += 1
                continue
            time.sleep(0.01)
        raise TimeoutError(f"peer {self.pid}: not admitted within {timeout_s}s")

    def leave(self):
        """Graceful leave: survivors drop this peer at their next round without a lease wait."""
        self.store.set(f"{_P}leave/{self.pid}", "1")
        self.stop_heartbeat()
        if self.group is not None:
            self.group.shutdown()
        self.group = None

    # ------------------------------------------------------------------ rounds
    def sync_round(self):
        """Barrier of the current generation. Returns (group, changed, newcomers).
        If this peer was voted out (arrived too late), it rejoins transparently."""
        self.round += 1
        k = self.round
        g = self.gen
        self.store.set(f"{_P}arrive/{g}/{k}/{self.pid}", "1")
        missing = [m for m in self.members if m != self.pid]
        hb_seen = {m: (self._hb(m), time.time()) for m in missing}
        dead, left = set(), set()
        t0 = time.time()
        nkey = f"{_P}gen/{g + 1}/members"
        while True:
            if self.store.check([nkey]):  # someone already decided the next generation
                return self._follow(g + 1, k)
            still = []
            for m in missing:
                if m in dead or m in left:
                    continue
                if self.store.check([f"{_P}arrive/{g}/{k}/{m}"]):
                    continue
                if self.store.check([f"{_P}leave/{m}"]):
                    left.add(m)
                    continue
                hb = self._hb(m)
                last, seen_at = hb_seen[m]
                if hb != last:
                    hb_seen[m] = (hb, time.time())
                elif time.time() - seen_at > self.lease_s:
                    dead.add(m)
                    continue
                still.append(m)
            missing_now = still
            njoin = self._njoin()
            if not missing_now:
                if not dead and not left and njoin <= self.joins_seen:
                    return self.group, False, []
                break
            if time.time() - t0 > self.arrive_timeout_s:
                dead.update(missing_now)
                break
            time.sleep(self.poll_s)
        # ---- propose the next generation: arrived members + pending joiners
        survivors = [m for m in self.members if m not in dead and m not in left]
        joiners = self._pending_joiners(njoin)
        proposal = sorted(set(survivors) | set(joiners))
        self.store.compare_set(f"{_P}gen/{g + 1}/joins", "", str(njoin))
        self.store.compare_set(nkey, "", ",".join(map(str, proposal)))
        return self._follow(g + 1, k)

    # ------------------------------------------------------------------ internals
    def _follow(self, g, k):
        members = [int(x) for x in _s(self.store.get(f"{_P}gen/{g}/members")).split(",") if x]
        old = set(self.members)
        if self.pid not in members:
            # voted out (late arrival): rejoin as a newcomer
            self.events.append({"event": "evicted", "gen": g})
            if self.group is not None:
                self.group.shutdown()
            self.group = None
            self.gen = g
            self.join()
            return self.group, True, [self.pid]
        self._adopt(g, members)
        newcomers = [m for m in members if m not in old]
        self.events.append({"event": "regroup", "gen": g, "members": members, "round": k,
                            "dropped": sorted(old - set(members)), "joined": newcomers})
        return self.group, True, newcomers

    def _adopt(self, g, members):
        if self.group is not None:
            self.group.shutdown()
        self.gen = g
        self.members = list(members)
        pk = f"{_P}gen/{g - 1}/members"
        if g > 0 and self.store.check([pk]):
            self.prev_members = [int(x) for x in _s(self.store.get(pk)).split(",") if x]
        else:
            self.prev_members = list(members)
        self.newcomers = [m for m in members if m not in self.prev_members]
        self.round = 0
        js = f"{_P}gen/{g}/joins"
        self.joins_seen = int(_s(self.store.get(js))) if self.store.check([js]) else self._njoin()
        self.group = PeerGroup(self.store, members.index(self.pid), len(members), self.backend, generation=g,
                               members=members, timeout_s=self.pg_timeout_s, device=self.device)

    def _hb(self, m) -> int:
        return int(self.store.add(f"{_P}hb/{m}", 0))

    def _njoin(self) -> int:
        return int(self.store.add(f"{_P}njoin", 0))

    def _pending_joiners(self, njoin):
        out = []
        for seq in range(self.joins_seen + 1, njoin + 1):
            key = f"{_P}join/{seq}"
            if self.store.check([key]):
                out.append(int(_s(self.store.get(key))))
        return out

    def _latest_gen(self) -> int:
        g = 0
        while self.store.check([f"{_P}gen/{g + 1}/members"]):
            g += 1
        return g if self.store.check([f"{_P}gen/{g}/members"]) else -1
