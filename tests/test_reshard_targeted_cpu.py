"""Targeted elastic re-shard of the ZeRO optimizer state (VERDICT r2 missing #4).

Four gloo peers train a few sharded steps (replicas = 1); then peer 3 leaves and the other three
re-shard onto a 3-peer layout. Every slice a peer holds afterwards (primary and replica: fp32
master, m, v) must equal the corresponding range of the global state from before, and the bytes
on the wire must be the changed slices only (each fetched once from one old holder), never the
full state (the previous scheme broadcast every shard to every peer and rebuilt the full
12 B/param state on each). Reference concept: the pool mutation on join/end
(/root/reference/server.py:104-109, 141-154).
"""
import torch

from tests import _mp

W = 4


def _body(rank, world, port):
    import datetime

    import torch.distributed as dist

    from distributedvolunteercomputing_amd.models.mlp import MLP, synthetic_mnist
    from distributedvolunteercomputing_amd.parallel.peer_group import PeerGroup
    from distributedvolunteercomputing_amd.parallel.zero import ShardedConfig, ShardedDPTrainer

    store = dist.TCPStore("127.0.0.1", port, None, rank == 0, timeout=datetime.timedelta(seconds=60),
                          wait_for_workers=False)
    g = PeerGroup(store, rank, world, "gloo", generation=0)
    tr = ShardedDPTrainer(MLP(seed=0), ShardedConfig(lr=1e-2, weight_decay=0.0, replicas=1), group=g, device="cpu")
    x, y = synthetic_mnist(128, seed=rank)
    for i in range(3):
        tr.step(x[i * 32:(i + 1) * 32], y[i * 32:(i + 1) * 32])
    n = tr.flat.numel
    # the global state before the regroup, from the primaries
    full = {}
    for f in ("master", "m", "v"):
        lo, hi = tr.prim
        buf = torch.zeros(n)
        buf[lo:hi] = getattr(tr, f)
        g.allreduce_(buf)
        full[f] = buf
    old_held = [tr.prim] + [r["range"] for r in tr.reps]
    params_before = tr.flat.param.clone()
    res = {"rank": rank}
    if rank < 3:
        ng = PeerGroup(store, rank, 3, "gloo", generation=1, members=[0, 1, 2])
        tr.reshard(ng)
        ev = tr.reshard_events[-1]
        held = [(tr.prim, tr.master, tr.m, tr.v)] + [(r["range"], r["master"], r["m"], r["v"]) for r in tr.reps]
        for (a, b), mm, m1, v1 in held:
            assert torch.equal(mm, full["master"][a:b]), (rank, a, b)
            assert torch.equal(m1, full["m"][a:b]) and torch.equal(v1, full["v"][a:b]), (rank, a, b)
        assert len(held) == 2  # primary + one replica on the 3-peer layout
        assert torch.equal(tr.flat.param, params_before)  # exact bf16 parameters kept
        # what this peer had to fetch: the elements of its new slices it did not hold before
        need = 0
        for (a, b), *_ in held:
            mask = torch.ones(b - a, dtype=torch.bool)
            for (c, d) in old_held:
                lo, hi = max(a, c), min(b, d)
                if hi > lo:
                    mask[lo - a:hi - a] = False
            need += int(mask.sum())
        res.update(sent=ev["bytes_sent"], changed=ev["bytes_changed"], need=12 * need, n=n)
        # one more step on the new layout works
        tr.step(x[96:128], y[96:128])
    return res


def test_targeted_reshard_moves_only_changed_slices():
    out = _mp.run(_body, W, timeout=120)
    sent = sum(out[r]["sent"] for r in range(3))
    changed = sum(out[r]["changed"] for r in range(3))
    need = sum(out[r]["need"] for r in range(3))
    n = out[0]["n"]
    assert changed == need  # each peer fetched exactly what it lacked
    assert sent == changed  # every changed byte crossed the wire once
    assert sent <= 2 * changed
    # far below the full-state broadcast of the previous scheme (3 peers x 12 B/param each)
    assert sent < 3 * 12 * n / 2, (sent, n)
