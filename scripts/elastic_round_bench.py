"""Host cost of one elastic round: P gloo peers on this host run
`sync_round()` + `guard()` around one tiny all-reduce, R times; printed is the mean wall time
per round against the same all-reduce without membership. The difference is the store traffic
(arrival record, agreement, verdict) that every training step pays.

    python scripts/elastic_round_bench.py [--peers 8] [--rounds 200]
"""
import argparse
import datetime
import json
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _peer(pid, port, P, R, q):
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch
    import torch.distributed as dist

    from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership

    torch.set_num_threads(1)
    store = dist.TCPStore("127.0.0.1", port, None, False, timeout=datetime.timedelta(seconds=120),
                          wait_for_workers=False)
    mem = ElasticMembership(store, pid, backend="gloo", lease_s=30.0, heartbeat_s=0.2)
    mem.bootstrap(list(range(P)))
    t = torch.ones(16)
    grp = mem.group
    grp.connect()
    for _ in range(10):
        grp.allreduce_(t)
    grp.barrier()
    t0 = time.perf_counter()
    for _ in range(R):
        grp.allreduce_(t)
    bare = (time.perf_counter() - t0) / R * 1e3
    grp.barrier()
    for _ in range(10):
        mem.sync_round()
        with mem.guard("s"):
            mem.group.allreduce_(t)
    mem.group.barrier()
    ops0 = getattr(mem, "store_ops", 0)
    t0 = time.perf_counter()
    for _ in range(R):
        mem.sync_round()
        with mem.guard("s"):
            mem.group.allreduce_(t)
    full = (time.perf_counter() - t0) / R * 1e3
    ops = (getattr(mem, "store_ops", 0) - ops0) / R
    mem.group.barrier()
    q.put((pid, bare, full, ops))
    mem.leave()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=200)
    a = ap.parse_args()
    import socket

    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore("127.0.0.1", port, None, True, timeout=datetime.timedelta(seconds=120),  # noqa: F841
                          wait_for_workers=False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_peer, args=(i, port, a.peers, a.rounds, q)) for i in range(a.peers)]
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join(60)
    bare = max(r[1] for r in res)
    full = max(r[2] for r in res)
    print(json.dumps({"peers": a.peers, "rounds": a.rounds, "allreduce_ms": round(bare, 3),
                      "round_ms": round(full, 3), "membership_overhead_ms": round(full - bare, 3),
                      "store_ops_per_round": round(max(r[3] for r in res), 1)}))


if __name__ == "__main__":
    main()
