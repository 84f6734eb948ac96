"""Elastic re-shard of sharded (ZeRO-1, replicas=1) Llama training on RCCL communicators, with a
peer SIGKILLed between steps.

Launched one process per peer (torchrun env) — on one MI355X through
scripts/rccl_rehearsal_launch.py --expect-killed <victim> (loopback-socket RCCL: the re-shard
time is a socket-transport number, not xGMI). Every peer bootstraps an ElasticMembership on a
TCPStore, trains `--steps` ShardedDPTrainer steps of a Llama-3 architecture on synthetic tokens,
and the victim SIGKILLs itself at `--kill-at`; the survivors detect the death on their liveness
links, regroup, re-shard the fp32 master/m/v point to point (only the slices that change holder
move) and keep training. Each survivor prints one JSON line: step times before/after, the
re-shard event (ms, bytes moved, bytes changed), and the peak HBM of its process.

Memory model for the verdict's 8B case (two peers, replicas=1): each peer then holds the WHOLE
fp32 state (its primary half + a replica of the other half, 12 B/param = 96 GB) plus bf16
params/grads (32 GB) and activations: ~135+ GB per peer, so two such peers cannot share one
288 GB card — this rehearsal runs the same code path on Llama-3.2-1B/3B-sized models instead.
"""
import argparse
import datetime
import json
import os
import signal
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.2-1b")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--kill-at", type=int, default=4)
    ap.add_argument("--victim", type=int, default=-1, help="rank that dies (default: the last)")
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--lease", type=float, default=2.0)
    ap.add_argument("--backend", default="nccl")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    victim = a.victim if a.victim >= 0 else world - 1
    import torch.distributed as dist

    from distributedvolunteercomputing_amd.models.llama import Llama, LlamaConfig
    from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership
    from distributedvolunteercomputing_amd.parallel.zero import ShardedConfig, ShardedDPTrainer

    dev = torch.device("cuda", 0) if a.backend == "nccl" else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    port = int(os.environ["MASTER_PORT"]) + 1
    store = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), port, None, rank == 0,
                          timeout=datetime.timedelta(seconds=300), wait_for_workers=False)
    mem = ElasticMembership(store, rank, backend=a.backend, device=dev if dev.type == "cuda" else None,
                            lease_s=a.lease, heartbeat_s=0.1)
    mem.bootstrap(list(range(world)))
    cfg = LlamaConfig.preset(a.model)
    model = Llama(cfg, seed=0).to(device=dev, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
    tr = ShardedDPTrainer(model, ShardedConfig(lr=1e-4, replicas=a.replicas), membership=mem, device=dev)
    g = torch.Generator().manual_seed(rank)
    toks = torch.randint(0, cfg.vocab_size, (a.batch, a.seq + 1), generator=g).to(dev)
    x, y = toks[:, :-1].contiguous(), toks[:, 1:].contiguous()
    times = []
    for i in range(a.steps):
        if rank == victim and i == a.kill_at:
            os.kill(os.getpid(), signal.SIGKILL)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss = tr.step(x, y)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    ev = tr.reshard_events[-1] if tr.reshard_events else {}
    out = {"rank": rank, "model": a.model, "params": tr.flat.numel, "peers_before": world, "peers_after": mem.group.size,
           "replicas": a.replicas, "gen": mem.gen, "loss": round(float(loss), 4),
           "step_ms": [round(t, 1) for t in times], "drop_step_ms": round(times[a.kill_at], 1),
           "reshard_ms": round(ev.get("ms", 0.0), 1), "reshard_bytes_sent": ev.get("bytes_sent"),
           "reshard_bytes_changed": ev.get("bytes_changed"), "state_bytes": tr.state_bytes(),
           "eof": [m for m, _ in mem.eof_events]}
    if dev.type == "cuda":
        out["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated() / 1e9, 2)
    print(json.dumps(out), flush=True)
    mem.leave()


if __name__ == "__main__":
    main()
