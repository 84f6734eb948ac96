"""Training peer: one process per GPU acting as an independent volunteer.

    python -m distributedvolunteercomputing_amd.cli.main train --model gpt2 --trainer localsgd --H 4 ...

Under torchrun (RANK/WORLD_SIZE/LOCAL_RANK set) every rank is a peer; otherwise pass
--peer-id/--world/--store-host/--store-port. With --elastic, membership runs through the
heartbeat/lease/generation protocol (parallel/elastic.py) on a TCPStore hosted by peer 0, so
peers may die (--drop-at: fault injection) and join or rejoin (--join) mid-training.

Models: mlp (synthetic MNIST), gpt2[-medium|-large|-xl|-tiny] (random tokens), resnet50 /
resnet-tiny (synthetic ImageNet), llama3-8b / llama3.2-1b / llama-tiny (random tokens).
Trainers: localsgd (H local AdamW steps + averaging) | sharded (ZeRO-1 + buddy replicas).
Compression: none | topk (ratio) | powersgd (rank). Checkpoints: utils/checkpoint.py format.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from .. import config


def build_model(name: str, device, seq: int):
    if name == "mlp":
        from ..models.mlp import MLP

        return MLP(), {"name": "mlp"}
    if name.startswith("gpt2"):
        from ..models.gpt2 import GPT2, GPT2Config

        cfg = GPT2Config.preset(name)
        cfg.n_ctx = max(cfg.n_ctx, seq)
        return GPT2(cfg), {"name": name, **cfg.__dict__}
    if name.startswith("resnet"):
        from ..models.resnet import resnet50, resnet_tiny

        return (resnet50() if name == "resnet50" else resnet_tiny()), {"name": name}
    if name.startswith("llama"):
        from ..models.llama import Llama, LlamaConfig

        cfg = LlamaConfig.preset(name)
        return Llama(cfg), {"name": name, **cfg.__dict__}
    raise ValueError(f"unknown model {name!r}")


class SyntheticData:
    def __init__(self, name, model, batch, seq, device, seed):
        self.name, self.batch, self.seq, self.device = name, batch, seq, device
        g = torch.Generator(device="cpu").manual_seed(seed)
        if name == "mlp":
            from ..models.mlp import synthetic_mnist

            self.x, self.y = synthetic_mnist(batch * 16, seed=seed, device=device)
        elif name.startswith("resnet"):
            n = 224 if name == "resnet50" else 32
            self.x = torch.randn(batch * 2, 3, n, n, generator=g).to(device, memory_format=torch.channels_last)
            nc = 1000 if name == "resnet50" else 10
            self.y = torch.randint(0, nc, (batch * 2,), generator=g).to(device)
        else:
            vocab = model.cfg.vocab_size if hasattr(model, "cfg") else model.c.vocab_size
            toks = torch.randint(0, vocab, (batch * 4, seq + 1), generator=g).to(device)
            self.x, self.y = toks[:, :-1], toks[:, 1:]

    def __call__(self, i):
        n = self.x.shape[0] // self.batch
        j = i % n
        sl = slice(j * self.batch, (j + 1) * self.batch)
        x = self.x[sl]
        if self.name.startswith("resnet"):
            x = x.to(torch.bfloat16) if self.device.type == "cuda" else x
        return x, self.y[sl]


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="train", description=__doc__.splitlines()[0])
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--trainer", default="localsgd", choices=["localsgd", "sharded"])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--H", type=int, default=4)
    ap.add_argument("--algo", default=None, choices=["rccl", "rs_ag", "butterfly", "ring", "direct", "rs"],
                    help="averaging collective (default: direct for localsgd, rs = reduce-scatter + replica "
                         "shifts for sharded)")
    ap.add_argument("--replicas", type=int, default=2, help="sharded: extra holders of every optimizer shard")
    ap.add_argument("--compression", default="none", choices=["none", "topk", "powersgd"])
    ap.add_argument("--topk-ratio", type=float, default=0.01)
    ap.add_argument("--powersgd-rank", type=int, default=4)
    ap.add_argument("--outer-lr", type=float, default=1.0)
    ap.add_argument("--outer-momentum", type=float, default=0.0)
    ap.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"])
    ap.add_argument("--elastic", action="store_true")
    ap.add_argument("--lease", type=float, default=5.0)
    ap.add_argument("--peer-id", type=int, default=None)
    ap.add_argument("--world", type=int, default=None)
    ap.add_argument("--store-host", default=os.environ.get("MASTER_ADDR", "127.0.0.1"))
    ap.add_argument("--store-port", type=int, default=config.get().store_port_train)
    ap.add_argument("--coordinator", default=None,
                    help="host:control_port of a coordinator that hosts the rendezvous store (no peer is special)")
    ap.add_argument("--train-token", default=os.environ.get("VCX_TRAIN_TOKEN"),
                    help="admission token for a coordinator started with one (tjoin)")
    ap.add_argument("--join", action="store_true", help="join a running job instead of bootstrapping")
    ap.add_argument("--drop-at", type=int, default=-1, help="fault injection: crash this peer at that step")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--metrics", default=None, help="JSONL metrics file")
    ap.add_argument("--trace-dir", default=config.get().trace_dir or None,
                    help="write per-stage device-time spans (HIP events) as JSONL here")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    rank = a.peer_id if a.peer_id is not None else int(os.environ.get("RANK", "0"))
    world = a.world if a.world is not None else int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", local % torch.cuda.device_count()) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    backend = a.backend or ("nccl" if cuda else "gloo")
    from ..parallel.peer_group import PeerGroup

    prefix = ""
    if a.coordinator:  # the coordinator hosts the rendezvous store: get admitted, learn where
        from ..control.protocol import ControlClient, split_store_ref

        host, _, cport = a.coordinator.rpartition(":")
        a.store_host = host
        ident = f"train-peer-{rank}" + (f"||{a.train_token}" if a.train_token else "")
        a.store_port, prefix = split_store_ref(ControlClient(host, int(cport)).call("tjoin", ident))
    store = dist.TCPStore(a.store_host, a.store_port, None, rank == 0 and not a.join and not a.coordinator,
                          timeout=datetime.timedelta(seconds=300), wait_for_workers=False)
    if prefix:  # every rendezvous key under the coordinator's secret prefix
        store = dist.PrefixStore(prefix, store)
    membership = group = None
    if a.elastic:
        from ..parallel.elastic import ElasticMembership, _route_ip

        membership = ElasticMembership(store, rank, backend=backend, device=device, lease_s=a.lease,
                                       live_host=_route_ip(a.store_host))
        if a.join:
            membership.join()
        else:
            membership.bootstrap(list(range(world)))
    elif world > 1:
        group = PeerGroup(store, rank, world, backend, device=device)

    torch.manual_seed(0)  # identical init on every peer
    model, mcfg = build_model(a.model, device, a.seq)
    dtype = torch.bfloat16 if cuda else torch.float32
    model = model.to(device=device, dtype=dtype)
    if a.model.startswith("resnet"):
        from ..models.resnet import enable_conv_find

        model = model.to(memory_format=torch.channels_last)
        if device.type == "cuda":
            enable_conv_find()
    if a.trainer == "localsgd":
        from ..parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

        cfg = LocalSGDConfig(lr=a.lr, H=a.H, algo=a.algo or "direct", outer_lr=a.outer_lr,
                             outer_momentum=a.outer_momentum,
                             comm_dtype=torch.bfloat16 if cuda else torch.float32)
        tr = LocalSGDTrainer(model, cfg, group=group, membership=membership, device=device)
    else:
        from ..parallel.zero import ShardedConfig, ShardedDPTrainer

        tr = ShardedDPTrainer(model, ShardedConfig(lr=a.lr, algo=a.algo or "rs", replicas=a.replicas), group=group,
                              membership=membership, device=device)
    if a.compression == "topk":
        from ..parallel.compression import TopKCompressor

        tr.compressor = TopKCompressor(tr.flat.numel, a.topk_ratio, device)
    elif a.compression == "powersgd":
        from ..parallel.compression import PowerSGDCompressor

        tr.compressor = PowerSGDCompressor(tr.flat, a.powersgd_rank, device)
    if a.join and membership is not None:
        tr.join_running_job()
    if a.resume and a.ckpt_dir:
        from ..utils.checkpoint import ShardReader, latest

        d = latest(a.ckpt_dir)
        if d:
            tr.restore(ShardReader(d))
            print(f"[peer {rank}] resumed from {d} at step {tr.t}", flush=True)

    tracer = None
    if a.trace_dir and hasattr(tr, "tracer"):
        from ..utils.trace import SpanTracer

        tracer = tr.tracer = SpanTracer(f"peer{rank}", path=os.path.join(a.trace_dir, f"peer{rank}.jsonl"))
    data = SyntheticData(a.model, model, a.batch, a.seq, device, seed=1000 + rank)
    log = open(a.metrics, "a") if a.metrics else None
    t_last = time.perf_counter()
    step = tr.t
    while step < a.steps:
        if step == a.drop_at:
            print(f"[peer {rank}] fault injection: crashing at step {step}", flush=True)
            if membership is not None:
                membership.stop_heartbeat()
            os._exit(0)
        x, y = data(step)
        out = tr.step(x, y)
        if tracer is not None and (step + 1) % a.log_every == 0:
            tracer.flush(step=step + 1, peer=rank)
        loss = out.extra["loss_t"] if hasattr(out, "extra") else out
        step += 1
        if a.ckpt_dir and a.ckpt_every and step % a.ckpt_every == 0 and (
                a.trainer == "sharded" or step % a.H == 0):
            from ..parallel.peer_group import PeerFailure
            from ..utils.checkpoint import save_checkpoint

            import contextlib

            g = tr.group
            try:
                # guarded like every other collective phase: a peer dying inside the checkpoint's
                # reduce-scatters / barrier aborts it within one lease (or at once through its
                # liveness link) instead of after the process-group timeout
                with (membership.guard("c") if membership is not None else contextlib.nullcontext()):
                    save_checkpoint(tr, a.ckpt_dir, step, peer_id=rank, is_writer=(g is None or g.rank == 0),
                                    members=(g.members if g is not None else [rank]),
                                    generation=(membership.gen if membership else 0), model_config=mcfg,
                                    barrier=(g.barrier if g is not None else None))
            except PeerFailure as e:  # a peer died mid-checkpoint: skip it, the next round regroups
                print(f"[peer {rank}] checkpoint at step {step} skipped: {e}", flush=True)
        if step % a.log_every == 0 or step == a.steps:
            if cuda:
                torch.cuda.synchronize()
            now = time.perf_counter()
            rec = {"peer": rank, "step": step, "loss": float(loss), "ms_per_step": (now - t_last) * 1e3 / a.log_every,
                   "members": (tr.group.size if tr.group is not None else 1),
                   "gen": membership.gen if membership else 0}
            t_last = now
            print(json.dumps(rec), flush=True)
            if log:
                log.write(json.dumps(rec) + "\n")
                log.flush()
    if membership is not None:
        membership.stop_heartbeat()
    return 0


if __name__ == "__main__":
    sys.exit(main())
