"""Staged admission (parallel/elastic.py, gloo groups): a joiner's generation is agreed one round
early and built during the local steps. Here a member dies in exactly that window -- after the
staged round committed, before the switch -- so the staged generation contains a dead member: the
switch's guard must trip, the survivors and the joiner recover to a generation without it, and
training goes on with every committed round identical on every peer that committed it."""
import hashlib
import multiprocessing as mp
import os
import queue as _q
import time
import traceback

import torch

from tests import _mp

W = 3
VICTIM = 2
JOINER = 3


def _store(port, master=False):
    import datetime

    import torch.distributed as dist

    return dist.TCPStore("127.0.0.1", port, None, master, timeout=datetime.timedelta(seconds=60),
                         wait_for_workers=False)


def _hash(t):
    return hashlib.sha1(t.detach().float().cpu().numpy().tobytes()).hexdigest()[:16]


def _peer(pid, port, q, join):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    try:
        torch.set_num_threads(1)
        q.put((pid, "ok", _body(pid, port, join)))
    except BaseException as e:  # noqa: BLE001
        q.put((pid, "err", f"{e!r}\n{traceback.format_exc()}"))


def _body(pid, port, join):
    from distributedvolunteercomputing_amd import config
    from distributedvolunteercomputing_amd.models.mlp import MLP, synthetic_mnist
    from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership
    from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

    config.update(elastic_stage_joins="gloo")
    store = _store(port)
    mem = ElasticMembership(store, pid, backend="gloo", lease_s=1.0, heartbeat_s=0.05, pg_timeout_s=30.0)
    if join:
        while not store.check(["go_join"]):
            time.sleep(0.01)
        mem.join()
    else:
        mem.bootstrap(list(range(W)))
    tr = LocalSGDTrainer(MLP(seed=0), LocalSGDConfig(H=2, lr=0.05, weight_decay=0.0, max_grad_norm=0.0,
                                                     comm_dtype=torch.float32), membership=mem, device="cpu")
    hist = {}
    if join:
        tr.join_running_job()
        hist[f"{mem.gen}/{mem.round}"] = _hash(tr.anchor)
    x, y = synthetic_mnist(256, seed=pid)
    i, last, t_end = 0, tr.sync_count, time.time() + 60
    while time.time() < t_end:
        if pid == VICTIM and mem._staged is not None:
            # the staged round has committed (the build starts after the commit): die before the switch
            os._exit(0)
        if pid == 0 and i == 6:
            store.set("go_join", "1")
        b = slice((i % 8) * 32, (i % 8 + 1) * 32)
        tr.step(x[b], y[b])
        i += 1
        if tr.sync_count != last:
            last = tr.sync_count
            hist[f"{mem.gen}/{mem.round}"] = _hash(tr.anchor)
        if store.check(["leaving"]):
            break
        members = set(mem.members)
        if JOINER in members and VICTIM not in members and mem.round >= 3:
            store.set("leaving", "1")
            break
    ev = [{k: e.get(k) for k in ("event", "gen", "members", "joined", "dropped", "round")} for e in mem.events]
    mem.leave()
    return {"hist": hist, "events": ev, "gen": mem.gen, "members": list(mem.members)}


def test_member_dies_between_staging_and_switch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _mp.free_port()
    store = _store(port, master=True)  # noqa: F841 — this process hosts the rendezvous
    procs = [ctx.Process(target=_peer, args=(pid, port, q, False), daemon=True) for pid in range(W)]
    procs.append(ctx.Process(target=_peer, args=(JOINER, port, q, True), daemon=True))
    for p in procs:
        p.start()
    out, errs, t0 = {}, [], time.time()
    try:
        while time.time() - t0 < 150 and len(out) + len(errs) < 3:  # peers 0, 1 and the joiner report
            try:
                pid, st, res = q.get(timeout=0.2)
            except _q.Empty:
                continue
            (out.__setitem__(pid, res) if st == "ok" else errs.append((pid, res)))
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    assert not errs, errs
    assert set(out) == {0, 1, JOINER}, (set(out), time.time() - t0)
    for pid, r in out.items():
        assert JOINER in r["members"] and VICTIM not in r["members"], (pid, r["members"])
    # the survivors staged the joiner's generation (with the victim still in it), then recovered
    staged = [e for e in out[0]["events"] if e["event"] == "staged"]
    assert staged and VICTIM in staged[0]["members"] and JOINER in staged[0]["members"], out[0]["events"]
    seen = {}
    for who, r in out.items():
        for key, h in r["hist"].items():
            seen.setdefault(key, {})[who] = h
    bad = {k: v for k, v in seen.items() if len(v) > 1 and len(set(v.values())) != 1}
    assert not bad, f"peers disagree after committed rounds: {bad}"
