"""Local-SGD training engine for volunteer peers (one process per GPU).

Each peer runs H local AdamW steps on its own data shard, then the peers average their model
(BASELINE.json configs 1, 2, 4: "local-SGD H=4 + butterfly all-reduce", "kill 2 then rejoin").

Per-step GPU work (all on the current HIP stream, graph-capturable):
  zero flat grad -> fwd/bwd -> [grad-norm kernel] -> AdamW prologue -> fused flat AdamW.
Every H steps (`sync`):
  membership round (elastic only) -> lsgd_delta kernel (bf16 pseudo-gradient)
  -> [compression: top-k+EF or PowerSGD] -> all-reduce SUM over live peers
  -> lsgd_apply kernel (average + optional outer Nesterov momentum, writes anchor/master/param).

Reference analog: the chunk (100 frames) is the reference's unit of independent work
(worker.py:16, server.py:77-91); here the unit is H optimizer steps.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import torch

from .. import ops
from ..utils.trace import NULL_TRACER
from .collectives import allreduce_sum_
from .flat_params import FlatParams


@dataclass
class LocalSGDConfig:
    lr: float = 6e-4
    betas: tuple = (0.9, 0.95)
    eps: float = 1e-8
    weight_decay: float = 0.1
    max_grad_norm: float = 1.0
    H: int = 4  # local steps between averaging rounds
    algo: str = "rccl"  # rccl | rs_ag | butterfly | ring
    outer_lr: float = 1.0
    outer_momentum: float = 0.0
    nesterov: bool = False
    comm_dtype: torch.dtype = torch.bfloat16
    compression: str = "none"  # none | topk | powersgd
    topk_ratio: float = 0.01
    powersgd_rank: int = 4


@dataclass
class StepStats:
    step: int
    loss: float | None
    synced: bool
    sync_ms: float = 0.0
    members: int = 1
    extra: dict = field(default_factory=dict)


class LocalSGDTrainer:
    def __init__(self, model: torch.nn.Module, cfg: LocalSGDConfig, *, group=None, membership=None,
                 device=None, compressor=None, tracer=None):
        self.model = model
        self.cfg = cfg
        self.device = device or next(model.parameters()).device
        self.flat = FlatParams(model, dtype=torch.bfloat16, device=self.device)
        n = self.flat.numel
        self.master = self.flat.param.float()
        self.m = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.v = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.anchor = self.master.clone()
        self.delta = torch.zeros(n, dtype=cfg.comm_dtype, device=self.device)
        self.outer_mom = torch.zeros(n, dtype=torch.float32, device=self.device) if cfg.outer_momentum > 0 else None
        self.ostate = ops.new_ostate(self.device, cfg.lr)
        self.membership = membership
        self.group = membership.group if membership is not None else group
        self.compressor = compressor
        self.tracer = tracer or NULL_TRACER  # utils/trace.py stage spans (HIP events)
        self.t = 0
        self.sync_count = 0
        self.last_sync_ms = 0.0

    # ------------------------------------------------------------------ per step
    def set_lr(self, lr: float):
        self.ostate[1].fill_(lr)

    def forward_backward(self, x, y):
        self.flat.zero_grad()
        loss = self.model(x, y)
        loss.backward()
        return loss

    def optimizer_step(self):
        c = self.cfg
        ops.adamw_step(self.flat.param, self.flat.grad, self.master, self.m, self.v, self.ostate,
                       n_decay=self.flat.n_decay, beta1=c.betas[0], beta2=c.betas[1], eps=c.eps,
                       wd=c.weight_decay, max_norm=c.max_grad_norm)

    # ------------------------------------------------------------------ hipGraph capture
    def capture(self, x, y, warmup: int = 3):
        """Capture zero-grad + forward + backward + fused AdamW of one local step into a
        hipGraph (torch.cuda.graph). Replays then cost one graph launch instead of ~300
        kernel launches; the averaging round stays outside the graph (collective,
        membership). x/y shapes are fixed from here on. Runs `warmup` real steps first."""
        assert x.is_cuda, "graph capture needs GPU tensors"
        self.graph = None
        self._gx = x.clone()
        self._gy = y.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):  # real steps (eager; an H boundary still averages)
                self.step(self._gx, self._gy)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        # thread_local: a process-group watchdog thread querying its events during capture
        # must not invalidate it
        with torch.cuda.graph(graph, capture_error_mode="thread_local"):
            self._gloss = self.forward_backward(self._gx, self._gy)
            self.optimizer_step()
        self.graph = graph
        return self

    def step(self, x, y) -> StepStats:
        tr = self.tracer
        if getattr(self, "graph", None) is not None:
            if x.data_ptr() != self._gx.data_ptr():
                self._gx.copy_(x, non_blocking=True)
                self._gy.copy_(y, non_blocking=True)
            with tr.span("local_step_graph"):
                self.graph.replay()
            loss = self._gloss
        else:
            with tr.span("fwd_bwd"):
                loss = self.forward_backward(x, y)
            with tr.span("adamw"):
                self.optimizer_step()
        self.t += 1
        synced = False
        if self.t % self.cfg.H == 0:
            with tr.span("average"):
                self.sync()
            synced = True
        return StepStats(self.t, None, synced, self.last_sync_ms, self.group.size if self.group else 1,
                         {"loss_t": loss.detach()})

    # ------------------------------------------------------------------ averaging
    def sync(self):
        t0 = time.perf_counter()
        newcomers = []
        if self.membership is not None:
            self.group, changed, newcomers = self.membership.sync_round()
            if changed and newcomers:
                self._admit_newcomers(newcomers)
        self._average(newcomers)
        self.sync_count += 1
        self.last_sync_ms = (time.perf_counter() - t0) * 1e3

    def _average(self, newcomers=()):
        g = self.group
        if g is not None and g.size > 1:
            ops.lsgd_delta(self.master, self.anchor, self.delta)
            contributors = g.size - len(newcomers)  # newcomers hold delta == 0
            if self.compressor is not None:
                avg = self.compressor.allreduce_mean(self.delta, g)
                scale = g.size / contributors
            else:
                allreduce_sum_(self.delta, g, self.cfg.algo)
                avg, scale = self.delta, 1.0 / contributors
            c = self.cfg
            ops.lsgd_apply(avg, self.anchor, self.master, self.flat.param, self.outer_mom, outer_lr=c.outer_lr,
                           mu=c.outer_momentum, nesterov=c.nesterov, avg_scale=scale)
        else:
            self.anchor.copy_(self.master)

    def _admit_newcomers(self, newcomers):
        """The new generation contains peers without the model: the first continuing member
        broadcasts the anchor (identical on all continuing members); newcomers adopt it as
        their weights. Continuing members keep their un-averaged local progress."""
        g = self.group
        members = g.members
        root = next(i for i, m in enumerate(members) if m not in newcomers)
        g.broadcast_(self.anchor, root=root)
        if self.outer_mom is not None:
            g.broadcast_(self.outer_mom, root=root)
        me = self.membership.pid if self.membership is not None else None
        if me in newcomers:
            self.master.copy_(self.anchor)
            ops.f32_to_bf16(self.anchor, self.flat.param)

    def join_running_job(self):
        """Called by a peer that was just admitted (``membership.join()``): receive the model
        and take part in the round that admitted it."""
        nc = self.membership.newcomers
        self._admit_newcomers(nc)
        self._average(nc)

    # ------------------------------------------------------------------ state
    def state_tensors(self):
        return {"master": self.master, "m": self.m, "v": self.v, "anchor": self.anchor, "ostate": self.ostate}

    def checkpoint_slice(self):
        """This peer's 1/P share of the (synchronised) state: call right after a sync round,
        when master == anchor on every peer. Moments are per-peer; each peer contributes its
        own slice of them."""
        P = 1 if self.group is None else self.group.size
        r = 0 if self.group is None else self.group.rank
        lo, hi = self.flat.shard_bounds(r, P)
        t = {"master": self.anchor[lo:hi], "m": self.m[lo:hi], "v": self.v[lo:hi]}
        if self.outer_mom is not None:
            t["outer_mom"] = self.outer_mom[lo:hi]
        return lo, hi, t

    def restore(self, reader):
        reader.check_layout(self.flat)
        n = self.flat.numel
        dev = self.device
        self.master.copy_(reader.read_range("master", 0, n).to(dev))
        self.anchor.copy_(self.master)
        self.m.copy_(reader.read_range("m", 0, n).to(dev))
        self.v.copy_(reader.read_range("v", 0, n).to(dev))
        if self.outer_mom is not None:
            self.outer_mom.copy_(reader.read_range("outer_mom", 0, n).to(dev))
        _, ost = reader.params()
        self.ostate.copy_(ost.to(dev))
        ops.f32_to_bf16(self.master, self.flat.param)
        self.t = reader.step
