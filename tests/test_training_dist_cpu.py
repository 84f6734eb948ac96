"""Multi-process CPU (gloo) tests of the training engines: local-SGD (BASELINE config 1),
compressed averaging, elastic drop/rejoin, ZeRO sharding with buddy re-shard."""
import os
import time

import pytest
import torch

from tests import _mp


def _mlp_trainer(rank, group=None, membership=None, H=2, compressor=None, lr=0.05):
    from distributedvolunteercomputing_amd.models.mlp import MLP
    from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

    m = MLP(seed=0)  # identical init on every peer
    cfg = LocalSGDConfig(H=H, lr=lr, weight_decay=0.0, max_grad_norm=0.0, comm_dtype=torch.float32
                         if compressor is None else torch.bfloat16)
    tr = LocalSGDTrainer(m, cfg, group=group, membership=membership, device="cpu")
    if compressor == "topk":
        from distributedvolunteercomputing_amd.parallel.compression import TopKCompressor

        tr.compressor = TopKCompressor(tr.flat.numel, 0.05, "cpu")
    elif compressor == "powersgd":
        from distributedvolunteercomputing_amd.parallel.compression import PowerSGDCompressor

        tr.compressor = PowerSGDCompressor(tr.flat, rank=4, device="cpu")
    return tr


def _local_sgd_worker(rank, world, port, algo, compressor):
    from distributedvolunteercomputing_amd.models.mlp import synthetic_mnist
    from distributedvolunteercomputing_amd.parallel.peer_group import PeerGroup

    store = _mp.make_store(rank, world, port)
    g = PeerGroup(store, rank, world, "gloo")
    tr = _mlp_trainer(rank, group=g, compressor=compressor)
    tr.cfg.algo = algo
    x, y = synthetic_mnist(512, seed=rank)
    losses = []
    for i in range(12):
        b = slice((i % 8) * 64, (i % 8 + 1) * 64)
        st = tr.step(x[b], y[b])
        losses.append(float(st.extra["loss_t"]))
    # all peers must hold bit-identical anchors after a sync round
    a = tr.anchor.clone()
    g.allreduce_(a)
    same = torch.allclose(a / world, tr.anchor, atol=1e-6)
    g.barrier()
    return {"first": losses[0], "last": losses[-1], "same": same, "syncs": tr.sync_count}


@pytest.mark.parametrize("algo", ["rccl", "butterfly"])
def test_local_sgd_two_peers_config1(algo):
    res = _mp.run(_local_sgd_worker, 2, algo, None)
    for r in res.values():
        assert r["same"] and r["syncs"] == 6
        assert r["last"] < r["first"] * 0.7, r


@pytest.mark.parametrize("comp", ["topk", "powersgd"])
def test_local_sgd_compressed(comp):
    res = _mp.run(_local_sgd_worker, 2, "rccl", comp)
    for r in res.values():
        assert r["same"]
        assert r["last"] < r["first"], r


def _elastic_worker(rank, world, port, drop_rank, rejoin):
    from distributedvolunteercomputing_amd.models.mlp import synthetic_mnist
    from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership

    store = _mp.make_store(rank, world, port)
    mem = ElasticMembership(store, rank, backend="gloo", lease_s=1.0, heartbeat_s=0.1)
    mem.bootstrap(list(range(world)))
    tr = _mlp_trainer(rank, membership=mem, H=2)
    x, y = synthetic_mnist(256, seed=rank)
    final_gen = 2 if rejoin else 1

    def run(tr, mem, i0):
        i = i0
        while not (mem.gen == final_gen and mem.round >= 2) and i < 2000:
            if mem.gen < final_gen and i > 200:
                time.sleep(0.01)  # waiting for the membership change: slow down, keep the rounds going
            b = slice((i % 8) * 32, (i % 8 + 1) * 32)
            tr.step(x[b], y[b])
            i += 1
            if rank == drop_rank and i == 5 and mem is first_mem:
                return i, True
        return i, False

    first_mem = mem
    i, dropped = run(tr, mem, 0)
    if dropped:
        mem.stop_heartbeat()  # simulated crash: vanish without a word
        if not rejoin:
            return {"dropped": True}
        time.sleep(2.0)
        mem = ElasticMembership(store, rank, backend="gloo", lease_s=1.0, heartbeat_s=0.1)
        mem.join()
        tr = _mlp_trainer(rank, membership=mem, H=2)
        tr.join_running_job()
        run(tr, mem, 0)
    store.set(f"done/{rank}", "1")
    if rank == 0:  # the store lives in rank 0: keep it up until every live peer is done
        live = [m for m in mem.members]
        t0 = time.time()
        while not store.check([f"done/{m}" for m in live]) and time.time() - t0 < 60:
            time.sleep(0.02)
    ev = [e for e in mem.events if e["event"] in ("regroup", "joined")]
    return {"members": mem.members, "events": ev, "anchor_sum": float(tr.anchor.sum()), "gen": mem.gen,
            "rejoined": dropped}


def test_elastic_drop_continues_on_survivors():
    res = _mp.run(_elastic_worker, 3, 2, False, timeout=120, expect_exit=(2,))
    for r in (0, 1):
        assert res[r]["members"] == [0, 1]
        assert any(e["dropped"] == [2] for e in res[r]["events"])
    assert abs(res[0]["anchor_sum"] - res[1]["anchor_sum"]) < 1e-4


def test_elastic_drop_and_rejoin():
    res = _mp.run(_elastic_worker, 3, 2, True, timeout=180)
    assert res[2]["rejoined"]
    # survivors went 3 -> 2 -> 3 peers
    for r in (0, 1):
        evs = res[r]["events"]
        assert any(e["dropped"] == [2] for e in evs) and any(e["joined"] == [2] for e in evs)


def _zero_worker(rank, world, port, drop_rank):
    from distributedvolunteercomputing_amd.models.mlp import MLP, synthetic_mnist
    from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership
    from distributedvolunteercomputing_amd.parallel.zero import ShardedConfig, ShardedDPTrainer

    store = _mp.make_store(rank, world, port)
    mem = ElasticMembership(store, rank, backend="gloo", lease_s=1.0, heartbeat_s=0.1)
    mem.bootstrap(list(range(world)))
    m = MLP(seed=0)
    tr = ShardedDPTrainer(m, ShardedConfig(lr=1e-2, weight_decay=0.0), membership=mem, device="cpu")
    x, y = synthetic_mnist(256, seed=rank)
    losses = []
    for i in range(10):
        if rank == drop_rank and i == 4:
            mem.stop_heartbeat()
            return {"dropped": True}
        losses.append(float(tr.step(x[i * 16:(i + 1) * 16], y[i * 16:(i + 1) * 16])))
    p = tr.flat.param.float().clone()
    mem.group.allreduce_(p)
    same = torch.allclose(p / mem.group.size, tr.flat.param.float(), atol=1e-6)
    return {"same": same, "members": mem.members, "lost": [e["lost"] for e in tr.reshard_events],
            "state_bytes": tr.state_bytes(), "first": losses[0], "last": losses[-1]}


def test_zero_sharded_buddy_reshard_after_drop():
    res = _mp.run(_zero_worker, 4, 3, timeout=180, expect_exit=(3,))
    for r in (0, 1, 2):
        assert res[r]["same"], res[r]
        assert res[r]["members"] == [0, 1, 2]
        assert res[r]["lost"] == [[]], res[r]["lost"]  # the dropped shard survived on its buddy
        assert res[r]["last"] < res[r]["first"]
