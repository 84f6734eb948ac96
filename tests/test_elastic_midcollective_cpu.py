"""Peers dying INSIDE a collective (BASELINE.json config 4: "kill 2 mid-training then rejoin").

Five gloo peers on CPU; the rendezvous store lives in this (parent) process, so any peer may
die. Two victims inject their own fault from inside a guarded collective (the PeerGroup fault
hook fires after the op was issued, while the other peers are blocked in it):

* SIGKILL: the victims vanish; the survivors' collective fails or their watchdog sees the
  leases expire, every survivor aborts the round, recovers to a new generation and redoes the
  round; fresh processes for the two victims then join the running job.
* SIGSTOP: the victims freeze mid-collective (no error on any socket: only the lease-based
  watchdog can notice); after the survivors regrouped, SIGCONT wakes them, they find their
  generation aborted, are evicted, and rejoin as newcomers in the same process.

Every peer records a hash of its averaged state after each committed round, keyed by
(generation, round); any two peers that committed the same round must hold identical state.
"""
import hashlib
import multiprocessing as mp
import os
import queue as _q
import signal
import time
import traceback

import pytest
import torch

from tests import _mp

W = 5
LEASE = 1.5


def _store(port, master=False):
    import datetime

    import torch.distributed as dist

    return dist.TCPStore("127.0.0.1", port, None, master, timeout=datetime.timedelta(seconds=120),
                         wait_for_workers=False)


def _hash(t):
    return hashlib.sha1(t.detach().float().cpu().numpy().tobytes()).hexdigest()[:16]


def _peer(pid, port, q, mode, kind, join, victims, n_rejoin, fault_op=None):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    try:
        torch.set_num_threads(1)
        res = _peer_body(pid, port, mode, kind, join, victims, n_rejoin, fault_op)
        q.put((pid, join, "ok", res))
    except BaseException as e:  # noqa: BLE001
        q.put((pid, join, "err", f"{e!r}\n{traceback.format_exc()}"))


def _peer_body(pid, port, mode, kind, join, victims, n_rejoin, fault_op_override=None):
    """A peer that, unless it is a victim, runs until both victims are back and it has
    committed 3 more rounds in the latest generation, recording a state hash per round."""
    from distributedvolunteercomputing_amd.models.mlp import MLP, synthetic_mnist
    from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership

    store = _store(port)
    mem = ElasticMembership(store, pid, backend="gloo", lease_s=LEASE, heartbeat_s=0.1, pg_timeout_s=30.0)
    fired = {"n": 0}
    model = MLP(seed=0)
    if mode == "lsgd":
        from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

        mk = lambda: LocalSGDTrainer(model, LocalSGDConfig(H=2, lr=0.05, weight_decay=0.0, max_grad_norm=0.0,  # noqa: E731
                                                           comm_dtype=torch.float32), membership=mem, device="cpu")
        fault_op, state = "alltoall", (lambda tr: tr.anchor)  # the direct all-reduce's first all-to-all
    else:
        from distributedvolunteercomputing_amd.parallel.zero import ShardedConfig, ShardedDPTrainer

        mk = lambda: ShardedDPTrainer(model, ShardedConfig(lr=1e-2, weight_decay=0.0, replicas=2),  # noqa: E731
                                      membership=mem, device="cpu")
        fault_op, state = "reduce_scatter", (lambda tr: tr.flat.param)
    fault_op = fault_op_override or fault_op

    if pid in victims and not join:
        def hook(grp, op):
            # the 3rd guarded gradient/averaging collective: every other member is inside it
            if op == fault_op:
                fired["n"] += 1
                if fired["n"] == 3:
                    os.kill(os.getpid(), signal.SIGKILL if kind == "kill" else signal.SIGSTOP)
        mem.fault_hook = hook
    if join:
        mem.join()
    else:
        mem.bootstrap(list(range(W)))
    tr = mk()
    hist = {}
    if join:
        tr.join_running_job()
        if mode == "lsgd":  # the admission round averaged too
            hist[f"{mem.gen}/{mem.round}"] = _hash(state(tr))
        store.add("rejoined", 1)
    x, y = synthetic_mnist(256, seed=pid)
    i, last_sync, rejoin_noted, t_end = 0, -1, join, time.time() + 90
    while time.time() < t_end:
        b = slice((i % 8) * 32, (i % 8 + 1) * 32)
        tr.step(x[b], y[b])
        i += 1
        synced = mode != "lsgd" or tr.sync_count != last_sync
        if mode == "lsgd":
            last_sync = tr.sync_count
        if synced and mem.group is not None:
            hist[f"{mem.gen}/{mem.round}"] = _hash(state(tr))
        if not rejoin_noted and any(e["event"] == "evicted" for e in mem.events):
            rejoin_noted = True  # stopped victim: woke up, found itself voted out, rejoined
            store.add("rejoined", 1)
        done = store.check(["leaving"]) or (int(store.add("rejoined", 0)) >= n_rejoin and mem.round >= 3
                                             and len(mem.members) == W)
        if done:
            store.set("leaving", "1")  # everyone winds down once the full group has run 3 rounds
            break
        time.sleep(0.003)
    ev = [e for e in mem.events if e["event"] in ("regroup", "joined", "evicted", "abort")]
    lost = [e["lost"] for e in getattr(tr, "reshard_events", [])]
    mem.leave()
    return {"hist": hist, "events": ev, "gen": mem.gen, "lost": lost,
            "failed": getattr(tr, "failed_rounds", getattr(tr, "failed_phases", 0))}


def _run(mode, kind, victims=(3, 4), timeout=150, fault_op=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _mp.free_port()
    store = _store(port, master=True)  # noqa: F841 — this process hosts the rendezvous
    n_rejoin = len(victims)
    procs = {pid: ctx.Process(target=_peer, args=(pid, port, q, mode, kind, False, victims, n_rejoin, fault_op),
                              daemon=True)
             for pid in range(W)}
    for p in procs.values():
        p.start()
    extra = []
    out, errs = {}, []
    t0 = time.time()
    respawned, conted = set(), False
    try:
        while time.time() - t0 < timeout:
            # controller: replace killed victims / wake stopped ones once the survivors regrouped
            for v in victims:
                p = procs[v]
                if kind == "kill" and v not in respawned and p.exitcode is not None:
                    assert p.exitcode == -signal.SIGKILL, p.exitcode
                    np_ = ctx.Process(target=_peer, args=(v, port, q, mode, kind, True, victims, n_rejoin), daemon=True)
                    np_.start()
                    extra.append(np_)
                    respawned.add(v)
            if kind == "stop" and not conted and _regrouped_without(store, victims):
                time.sleep(0.5)
                for v in victims:
                    os.kill(procs[v].pid, signal.SIGCONT)
                conted = True
            need = {(pid, False) for pid in range(W) if not (kind == "kill" and pid in victims)}
            need |= {(v, True) for v in victims} if kind == "kill" else set()
            if need.issubset(set(out) | {k for k, _ in errs}):
                break
            try:
                pid, join, st, res = q.get(timeout=0.2)
            except _q.Empty:
                continue
            if st == "ok":
                out[(pid, join)] = res
            else:
                errs.append(((pid, join), res))
    finally:
        for p in list(procs.values()) + extra:
            if p.is_alive():
                try:
                    os.kill(p.pid, signal.SIGCONT)
                except ProcessLookupError:
                    pass
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    if errs:
        raise AssertionError("peer failures:\n" + "\n".join(f"[{k}] {e}" for k, e in errs))
    return out


def _regrouped_without(store, victims):
    k = "vcx/el/gen/1"
    if not store.check([k]):
        return False
    members = [int(x) for x in store.get(k).decode().split("|")[0].split(",") if x]
    return not set(victims) & set(members)


def _check_consistent(out):
    seen = {}
    for who, r in out.items():
        for key, h in r["hist"].items():
            seen.setdefault(key, {})[who] = h
    shared = {k: v for k, v in seen.items() if len(v) > 1}
    bad = {k: v for k, v in shared.items() if len(set(v.values())) != 1}
    assert not bad, f"peers disagree after committed rounds: {bad}"
    return shared


def _assert_recovered(out, victims):
    survivors = [(p, False) for p in range(W) if p not in victims]
    for s in survivors:
        r = out[s]
        # each victim's old instance left the group: dropped by lease, or (when its replacement
        # registered before the survivors decided) replaced by the new instance in one regroup
        gone = {x for e in r["events"] if e["event"] == "regroup" for x in e["dropped"] + e["joined"]}
        assert set(victims) <= gone, r["events"]
        assert any(e["event"] == "abort" for e in r["events"]), "the failure must hit inside a collective"
        joined = {x for e in r["events"] if e["event"] == "regroup" for x in e["joined"]}
        assert set(victims) <= joined, r["events"]
        assert r["failed"] >= 1


@pytest.mark.parametrize("kind", ["kill", "stop"])
def test_localsgd_two_peers_die_inside_allreduce_then_rejoin(kind):
    victims = (3, 4)
    out = _run("lsgd", kind, victims)
    _assert_recovered(out, victims)
    shared = _check_consistent(out)
    # the rejoined victims committed rounds together with the survivors
    for v in victims:
        who = (v, kind == "kill")
        late = [k for k in out[who]["hist"] if int(k.split("/")[0]) >= 2]
        assert any(len(shared.get(k, {})) >= 3 for k in late), (who, out[who]["hist"])


@pytest.mark.parametrize("fault_op", ["reduce_scatter", "all_gather"])
def test_sharded_two_adjacent_peers_killed_inside_a_phase_no_state_lost(fault_op):
    """reduce_scatter: the gradient phase; all_gather: the parameter phase, while the victims'
    replacements register as joiners (after a parameter-phase recovery the survivors
    and a peer admitted in it must enter the same next phase)."""
    victims = (2, 3)  # adjacent: shard 2's primary and first replica die together
    out = _run("zero", "kill", victims, fault_op=fault_op)
    _assert_recovered(out, victims)
    _check_consistent(out)
    for who, r in out.items():
        for lost in r["lost"]:
            assert lost == [], (who, r["lost"])
