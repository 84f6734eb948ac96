"""Sharded data-parallel training: ZeRO-1 optimizer-state sharding across volunteer peers,
buddy replication of every shard, optional gradient compression, elastic re-shard.

Per step (all on the GPU stream):
  fwd/bwd -> flat bf16 grads -> average over live peers (RCCL all-reduce, or PowerSGD /
  top-k with error feedback) -> grad-norm kernel -> fused AdamW on MY shard and on my
  left neighbour's shard (the buddy replica) -> all-gather of the updated bf16 param shards.

Fault tolerance: shard j is held by peer j (primary) and peer j+1 (buddy). Because every
peer has the full averaged gradient after the all-reduce, the buddy applies the very same
AdamW update to its replica — no extra traffic per step; only 2x the (HBM-bound) optimizer
work on 2/P of the model. When a peer drops, its shard survives on its buddy; when the
membership changes the survivors re-shard by rebuilding the full fp32 optimizer state once
(affordable inside 288 GB of HBM: 12 B/param, 96 GB for an 8B model) from the live holders
and slicing the new primary/buddy ranges out of it.

No reference analog: SURVEY.md §2.7 "Optimizer-state sharding (ZeRO-like)" and §2.9
"Optimizer-state sharding + elastic re-shard" (BASELINE.json configs 4 and 5).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from .. import ops
from ..ops.optim import OS_SUMSQ
from .collectives import allreduce_sum_
from .flat_params import FlatParams


@dataclass
class ShardedConfig:
    lr: float = 3e-4
    betas: tuple = (0.9, 0.95)
    eps: float = 1e-8
    weight_decay: float = 0.1
    max_grad_norm: float = 1.0
    replicate: bool = True  # keep a buddy replica of the left neighbour's shard
    algo: str = "rccl"


class ShardedDPTrainer:
    def __init__(self, model, cfg: ShardedConfig, *, group=None, membership=None, compressor=None, device=None):
        self.model = model
        self.cfg = cfg
        self.device = torch.device(device or next(model.parameters()).device)
        self.flat = FlatParams(model, device=self.device)
        self.membership = membership
        self.group = membership.group if membership is not None else group
        self.compressor = compressor
        self.ostate = ops.new_ostate(self.device, cfg.lr)
        self.t = 0
        self.reshard_events = []
        self._layout(full_master=self.flat.param.float(), full_m=None, full_v=None)

    # ------------------------------------------------------------------ layout
    @property
    def world(self):
        return 1 if self.group is None else self.group.size

    @property
    def rank(self):
        return 0 if self.group is None else self.group.rank

    def _slices(self):
        P, r = self.world, self.rank
        prim = self.flat.shard_bounds(r, P)
        back = self.flat.shard_bounds((r - 1) % P, P) if (self.cfg.replicate and P > 1) else None
        return prim, back

    def _layout(self, full_master, full_m, full_v):
        (lo, hi), back = self._slices()
        self.prim = (lo, hi)
        self.back = back

        def cut(full, a, b):
            if full is None:
                return torch.zeros(b - a, dtype=torch.float32, device=self.device)
            return full[a:b].clone()

        self.master = cut(full_master, lo, hi)
        self.m = cut(full_m, lo, hi)
        self.v = cut(full_v, lo, hi)
        if back is not None:
            a, b = back
            self.b_master, self.b_m, self.b_v = cut(full_master, a, b), cut(full_m, a, b), cut(full_v, a, b)
        else:
            self.b_master = self.b_m = self.b_v = None

    def checkpoint_slice(self):
        lo, hi = self.prim
        return lo, hi, {"master": self.master, "m": self.m, "v": self.v}

    def restore(self, reader):
        """Load a checkpoint written by any number of peers into the CURRENT layout."""
        reader.check_layout(self.flat)
        dev = self.device
        param, ost = reader.params()
        self.flat.param.copy_(param.to(dev))
        self.ostate.copy_(ost.to(dev))
        lo, hi = self.prim
        self.master.copy_(reader.read_range("master", lo, hi).to(dev))
        self.m.copy_(reader.read_range("m", lo, hi).to(dev))
        self.v.copy_(reader.read_range("v", lo, hi).to(dev))
        if self.back is not None:
            a, b = self.back
            self.b_master.copy_(reader.read_range("master", a, b).to(dev))
            self.b_m.copy_(reader.read_range("m", a, b).to(dev))
            self.b_v.copy_(reader.read_range("v", a, b).to(dev))
        self.t = reader.step

    def state_bytes(self) -> int:
        n = self.master.numel() + (self.b_master.numel() if self.b_master is not None else 0)
        return 12 * n

    # ------------------------------------------------------------------ step
    def step(self, x, y):
        if self.membership is not None:
            grp, changed, newcomers = self.membership.sync_round()
            if changed:
                self.reshard(grp, old_members=self.membership.prev_members)
        self.flat.zero_grad()
        loss = self.model(x, y)
        loss.backward()
        g = self.flat.grad
        P = self.world
        if self.compressor is not None:
            avg = self.compressor.allreduce_mean(g, self.group)
        else:
            allreduce_sum_(g, self.group, self.cfg.algo)
            if P > 1:
                g.div_(P)
            avg = g
        self._adam(avg)
        self._gather_params()
        self.t += 1
        return loss.detach()

    def _adam_range(self, avg, a, b, master, m, v):
        c = self.cfg
        n_decay = max(0, min(self.flat.n_decay - a, b - a))
        n_decay -= n_decay % 8
        # the flat kernels read ostate (step/lr/clip) — shared by both ranges, prologue once
        C = ops.native() if self.flat.param.is_cuda else None
        if C is not None:
            C.adamw_flat(self.flat.param[a:b], avg[a:b], master, m, v, n_decay, self.ostate, c.betas[0], c.betas[1],
                         c.eps, c.weight_decay)
        else:
            from ..ops.optim import adamw_step

            st = self.ostate.clone()
            st[0] -= 1  # the reference increments step itself
            adamw_step(self.flat.param[a:b], avg[a:b], master, m, v, st, n_decay=n_decay, beta1=c.betas[0],
                       beta2=c.betas[1], eps=c.eps, wd=c.weight_decay, max_norm=0.0)

    def _adam(self, avg):
        c = self.cfg
        if avg.is_cuda:
            C = ops.native()
            if c.max_grad_norm > 0:
                self.ostate[OS_SUMSQ].zero_()
                C.grad_sumsq(avg, self.ostate)
            C.adam_prologue(self.ostate, float(c.max_grad_norm))
        else:
            self.ostate[0] += 1
            coef = 1.0
            if c.max_grad_norm > 0:
                nrm = avg.float().norm().item()
                coef = min(1.0, c.max_grad_norm / (nrm + 1e-6))
            self.ostate[2] = coef
            if coef != 1.0:
                avg = (avg.float() * coef).to(avg.dtype)
                self.ostate[2] = 1.0
        lo, hi = self.prim
        self._adam_range(avg, lo, hi, self.master, self.m, self.v)
        if self.back is not None:
            a, b = self.back
            self._adam_range(avg, a, b, self.b_master, self.b_m, self.b_v)

    def _gather_params(self):
        if self.world == 1:
            return
        lo, hi = self.prim
        mine = self.flat.param[lo:hi].clone()
        self.group.all_gather_(self.flat.param, mine)

    # ------------------------------------------------------------------ elastic re-shard
    def join_running_job(self):
        """A newly admitted peer takes part in the re-shard that admitted it (it holds no
        shard, so it only receives)."""
        self.reshard(self.membership.group, old_members=self.membership.prev_members)

    def reshard(self, new_group, old_members=None):
        """Membership changed: rebuild the full optimizer state from the live holders of every
        old shard (primary, else its buddy), then cut the new primary/buddy slices."""
        t0 = time.perf_counter()
        if old_members is None:
            old_members = list(self.group.members) if self.group is not None else [self.membership.pid]
        old_P = len(old_members)
        mine_old = self.prim
        back_old = self.back
        my_pid = self.membership.pid if self.membership is not None else self.rank
        self.group = new_group
        new_members = list(new_group.members)
        n = self.flat.numel
        full = [torch.zeros(n, dtype=torch.float32, device=self.device) for _ in range(3)]
        lost = []
        for j, owner in enumerate(old_members):
            a, b = self.flat.shard_bounds(j, old_P)
            if b <= a:
                continue
            buddy = old_members[(j + 1) % old_P] if (self.cfg.replicate and old_P > 1) else None
            if owner in new_members:
                holder, src = owner, "prim"
            elif buddy is not None and buddy in new_members:
                holder, src = buddy, "back"
            else:
                lost.append((a, b))
                continue
            root = new_members.index(holder)
            if holder == my_pid:
                bufs = (self.master, self.m, self.v) if src == "prim" else (self.b_master, self.b_m, self.b_v)
                assert (mine_old if src == "prim" else back_old) == (a, b)
                for f, s in zip(full, bufs):
                    f[a:b].copy_(s)
            for f in full:
                new_group.broadcast_(f[a:b], root=root) if new_group.size > 1 else None
        for a, b in lost:  # no live replica: restart that range from the current bf16 params
            full[0][a:b].copy_(self.flat.param[a:b].float())
        # joiners (and everybody) now hold the full fp32 master: refresh the bf16 params from it
        ops.f32_to_bf16(full[0], self.flat.param)
        if new_group.size > 1:  # ostate (step counter / lr) must agree across peers
            new_group.broadcast_(self.ostate, root=0)
        self._layout(*full)
        del full
        self.reshard_events.append({"t": self.t, "old": old_members, "new": new_members, "lost": lost,
                                    "ms": (time.perf_counter() - t0) * 1e3})
