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
from .flat_params import FlatBuffers, FlatParams
from .peer_group import PeerFailure


@dataclass
class LocalSGDConfig:
    lr: float = 6e-4
    betas: tuple = (0.9, 0.95)
    eps: float = 1e-8
    weight_decay: float = 0.1
    max_grad_norm: float = 1.0
    H: int = 4  # local steps between averaging rounds
    algo: str = "direct"  # direct | rccl | rs_ag | butterfly | ring (parallel/collectives.py)
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
        self.buffers = FlatBuffers(model)  # BN running stats: averaged at every sync
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
        self.t_sync_end = None
        self.failed_rounds = 0  # elastic rounds aborted mid-collective and redone
        self.admit_split = None  # the last admission transfer: communicator init vs broadcast (ms, bytes)
        self.last_round_stages = None  # a continuing member's stages of the last admission round
        # bench.py: time the averaging collective alone (device-synchronised on both sides) and
        # record its bytes, for algbw / busbw in the bench JSON
        self.time_reduce = False
        self.reduce_log: list[tuple[float, int]] = []  # (ms, bytes per rank) of each timed collective

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
        if self.membership is None:
            res = self._reduce(())
            self._apply(res)
            self.buffers.average_(self.group)
        else:
            self._sync_elastic()
        self.sync_count += 1
        self.last_sync_ms = (time.perf_counter() - t0) * 1e3
        self.t_sync_end = time.time()

    def _sync_elastic(self):
        """One elastic averaging round: agreed outcome -> guarded admission + reduction ->
        agreed verdict -> apply. A member dying inside the collectives aborts the round on
        every survivor; they restore the pre-round state (anchor/master were never touched,
        the pseudo-gradient is recomputed, the compressor state is rolled back) and redo the
        round on the next generation."""
        mem = self.membership
        t0 = time.perf_counter()
        grp, _, newcomers = mem.sync_round()
        t1 = time.perf_counter()
        self.last_round_stages = None
        while True:
            self.group = grp
            snap = self.compressor.snapshot() if (self.compressor is not None and grp.size > 1) else None
            try:
                with mem.guard():
                    t2 = time.perf_counter()
                    adopted = self._admit_newcomers(newcomers) if newcomers else None
                    self._dev_sync()
                    t3 = time.perf_counter()
                    res = self._reduce(newcomers)
                    bufs = self.buffers.averaged(grp)
                    self._dev_sync()
                    t4 = time.perf_counter()
                self._adopt(adopted)  # nothing is applied before the verdict is `commit`
                self._apply(res, bufs)
                if newcomers:
                    # a continuing member's anatomy of an admission round (where the
                    # members' rejoin stall goes): membership agreement, the new group's first
                    # collective (RCCL communicator init), the model broadcast, the reduction, and
                    # what is left (guard entry / exit, verdict, apply)
                    self._dev_sync()
                    t5 = time.perf_counter()
                    ad = self.admit_split or {}
                    self.last_round_stages = {
                        "sync_round_ms": round((t1 - t0) * 1e3, 3),
                        "peer_wait_ms": round(ad.get("peer_wait_ms", 0.0), 3),
                        "comm_init_ms": round(ad.get("comm_init_ms", 0.0), 3),
                        "broadcast_ms": round(ad.get("broadcast_ms", 0.0), 3),
                        "reduce_ms": round((t4 - t3) * 1e3, 3),
                        "guard_verdict_apply_ms": round(((t5 - t1) - (t4 - t2)) * 1e3, 3),
                        "broadcast_bytes": ad.get("bytes", 0),
                    }
                return
            except PeerFailure:
                if snap is not None:
                    self.compressor.restore(snap)
                # an abandoned gloo op may still own the old pseudo-gradient buffer
                self.delta = torch.zeros_like(self.delta)
                self.failed_rounds += 1
                grp, _, newcomers = mem.recover()

    def _reduce(self, newcomers=()):
        """Pseudo-gradient + collective. Returns what `_apply` needs; touches no model state."""
        g = self.group
        if g is None or g.size == 1:
            return None
        ops.lsgd_delta(self.master, self.anchor, self.delta)
        contributors = max(1, g.size - len(newcomers))  # newcomers hold delta == 0
        if self.compressor is not None:
            avg = self.compressor.allreduce_mean(self.delta, g)
            return avg, g.size / contributors
        if self.time_reduce:
            self._dev_sync()
            t0 = time.perf_counter()
        allreduce_sum_(self.delta, g, self.cfg.algo)
        if self.time_reduce:
            self._dev_sync()
            self.reduce_log.append(((time.perf_counter() - t0) * 1e3, self.delta.numel() * self.delta.element_size()))
        return self.delta, 1.0 / contributors

    def _apply(self, res, bufs=None):
        if bufs is not None:
            self.buffers.load_fp32(bufs)
        if res is None:
            self.anchor.copy_(self.master)
            return
        avg, scale = res
        c = self.cfg
        ops.lsgd_apply(avg, self.anchor, self.master, self.flat.param, self.outer_mom, outer_lr=c.outer_lr,
                       mu=c.outer_momentum, nesterov=c.nesterov, avg_scale=scale)

    def _average(self, newcomers=()):
        self._apply(self._reduce(newcomers))

    def _admit_newcomers(self, newcomers):
        """The generation contains peers without the model (joiners, or members whose earlier
        admission was aborted): the first continuing member broadcasts ONE packed fp32 vector
        [anchor | outer momentum | BN buffers] (identical on every continuing member) to the whole
        group, so every newcomer gets it in one pipelined collective instead of one point-to-point
        transfer per newcomer from the same root (RCCL: ring/tree broadcast over the xGMI links).
        Everyone receives into scratch; a newcomer adopts the model only after the round's verdict
        is `commit` (``_adopt``), so an aborted transfer can never corrupt any peer.
        Returns what the newcomer adopts (None on continuing members)."""
        g = self.group
        members = g.members
        cont = [i for i, m in enumerate(members) if m not in newcomers]
        if not cont:
            return None  # nobody holds a model yet: everyone starts from its own (identical) init
        root = cont[0]
        dev = self.anchor.device
        parts = [self.anchor] + ([self.outer_mom] if self.outer_mom is not None else [])
        nb = self.buffers.numel if self.buffers else 0
        n = sum(p.numel() for p in parts) + nb
        bdev = dev if g.backend == "nccl" else torch.device("cpu")
        if g.rank == root:
            pack = torch.cat([p.reshape(-1).to(bdev) for p in parts]
                             + ([self.buffers.as_fp32().to(bdev)] if nb else []))
        else:
            pack = torch.empty(n, dtype=torch.float32, device=bdev)
        # every member of the new group checks in at the rendezvous store first, so the communicator
        # set-up below is timed from the moment the LAST rank arrived: a member that enters the admission
        # round while a joiner is still starting up waits here (peer_wait_ms), not inside the init
        # (the members' 2.56 s vs the joiners' 1.34 s of "communicator init")
        tw = time.perf_counter()
        self._admission_checkin(g)
        # a one-element collective first: its time is the new group's communicator set-up (RCCL builds
        # its communicator lazily, at the first collective) plus one latency, so the broadcast time
        # below is the model transfer alone
        t0 = time.perf_counter()
        g.broadcast_(torch.zeros(1, dtype=torch.float32, device=bdev), root)
        self._dev_sync()
        t1 = time.perf_counter()
        g.broadcast_(pack, root)
        self._dev_sync()
        t2 = time.perf_counter()
        self.admit_split = {"peer_wait_ms": (t0 - tw) * 1e3, "comm_init_ms": (t1 - t0) * 1e3,
                            "broadcast_ms": (t2 - t1) * 1e3, "bytes": int(n * 4)}
        return pack if members[g.rank] in newcomers else None

    def _admission_checkin(self, g):
        """Store barrier of the admission round's group (elastic runs only): add one to the generation's
        check-in counter and wait until every member has; a trip of the watchdog (a member died) ends
        the wait as a PeerFailure like any guarded collective."""
        mem = self.membership
        if mem is None or g.size <= 1:
            return
        key = f"vcx/el/admit_in/{mem.gen}"
        mem.store.add(key, 1)
        while int(mem.store.add(key, 0)) < g.size:
            if mem.tripped():
                raise PeerFailure(f"gen {mem.gen}: aborted during the admission check-in ({mem.abort_reason()})")
            time.sleep(0.001)

    def _dev_sync(self):
        if self.anchor.is_cuda:
            torch.cuda.synchronize(self.anchor.device)

    def _adopt(self, pack):
        """A newcomer takes the admitted model (after `commit`)."""
        if pack is None:
            return
        pack = pack.to(self.anchor.device)
        n0 = self.anchor.numel()
        self.anchor.copy_(pack[:n0])
        pos = n0
        if self.outer_mom is not None:
            self.outer_mom.copy_(pack[pos:pos + n0])
            pos += n0
        if self.buffers:
            self.buffers.load_fp32(pack[pos:pos + self.buffers.numel])
        self.master.copy_(self.anchor)
        ops.f32_to_bf16(self.anchor, self.flat.param)

    def join_running_job(self):
        """Called by a peer that was just admitted (``membership.join()``): receive the model
        and take part in the round that admitted it (retried on the next generation if a
        member dies during it)."""
        mem = self.membership
        grp, newcomers = mem.group, mem.newcomers
        dev_sync = (lambda: torch.cuda.synchronize(self.anchor.device)) if self.anchor.is_cuda else (lambda: None)
        while True:
            self.group = grp
            try:
                # stage times of the admission (bench_drop.py reports them): communicator connect,
                # the wait for the members to enter the admission round (staged admission: they
                # finish their local steps first), then the round itself -- model broadcast,
                # reduction, verdict + apply
                t0 = time.perf_counter()
                with mem.guard():  # connect, then line up with the continuing members (wait_round_start)
                    dev_sync()
                    t2 = time.perf_counter()
                    t1 = t2 - mem.last_go_wait_ms * 1e-3
                    adopted = self._admit_newcomers(newcomers)
                    dev_sync()
                    t3 = time.perf_counter()
                    res = self._reduce(newcomers)
                    bufs = self.buffers.averaged(grp)
                    dev_sync()
                    t4 = time.perf_counter()
                self._adopt(adopted)
                self._apply(res, bufs)
                dev_sync()
                t5 = time.perf_counter()
                ad = self.admit_split or {}
                st = {"connect_ms": (t1 - t0) * 1e3, "wait_round_ms": (t2 - t1) * 1e3,
                      "peer_wait_ms": ad.get("peer_wait_ms", 0.0), "comm_init_ms": ad.get("comm_init_ms", 0.0), "broadcast_ms": ad.get("broadcast_ms", (t3 - t2) * 1e3),
                      "reduce_ms": (t4 - t3) * 1e3,
                      "verdict_apply_ms": (t5 - t4) * 1e3, "admission_round_ms": (t5 - t2) * 1e3,
                      "broadcast_bytes": ad.get("bytes", int(self.anchor.numel() * 4 * (2 if self.outer_mom is not None else 1)))}
                self.admit_stages = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in st.items()}
                return
            except PeerFailure:
                self.delta = torch.zeros_like(self.delta)
                self.failed_rounds += 1
                grp, _, newcomers = mem.recover()

    # ------------------------------------------------------------------ state
    def state_tensors(self):
        return {"master": self.master, "m": self.m, "v": self.v, "anchor": self.anchor, "ostate": self.ostate}

    def checkpoint_slice(self):
        """This peer's 1/P share of the (synchronised) state: call right after a sync round,
        when master == anchor on every peer. Adam moments and the compressor's error feedback
        are per-peer; the checkpoint stores their mean over the peers (one reduce-scatter each,
        so every peer writes the averaged slice it owns) — a restore onto any peer count then
        starts every peer from the same coherent moments, and from the mean unsent residual
        (exactly what the next averaging round would have delivered)."""
        P = 1 if self.group is None else self.group.size
        r = 0 if self.group is None else self.group.rank
        lo, hi = self.flat.shard_bounds(r, P)
        t = {"master": self.anchor[lo:hi], "m": mean_slice(self.group, self.m, lo, hi),
             "v": mean_slice(self.group, self.v, lo, hi)}
        if self.outer_mom is not None:
            t["outer_mom"] = self.outer_mom[lo:hi]  # identical on every peer (updated from the average)
        if self.compressor is not None:
            t["ef"] = mean_slice(self.group, self.compressor.state_dict()["ef"], lo, hi)
        return lo, hi, t

    def checkpoint_global(self) -> dict:
        """Tensors written once (by the writer peer) next to the parameters."""
        out = {}
        if self.buffers:
            out["buffers"] = self.buffers.as_fp32()
        if self.compressor is not None and "Q" in self.compressor.state_dict():
            out["psgd_Q"] = self.compressor.state_dict()["Q"]  # identical on every peer (all-reduced)
        return out

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
        restore_extras(self, reader)
        self.t = reader.step


def mean_slice(group, buf, lo, hi):
    """[lo, hi) of the peers' mean of `buf` (this peer's shard): one reduce-scatter."""
    if group is None or group.size == 1:
        return buf[lo:hi]
    P = group.size
    if buf.numel() % P == 0 and hi - lo == buf.numel() // P:
        out = torch.empty(hi - lo, dtype=buf.dtype, device=buf.device)
        group.reduce_scatter_(out, buf)
    else:
        tmp = buf.clone()
        group.allreduce_(tmp)
        out = tmp[lo:hi]
    return out.div_(P)


def restore_extras(trainer, reader):
    """BN buffers and compressor state (error feedback, PowerSGD's Q) if the checkpoint has them."""
    bufs = reader.global_tensor("buffers")
    if bufs is not None and trainer.buffers:
        trainer.buffers.load_fp32(bufs)
    comp = trainer.compressor
    if comp is not None and reader.has_key("ef"):
        d = {"ef": reader.read_range("ef", 0, trainer.flat.numel)}
        q = reader.global_tensor("psgd_Q")
        if q is not None:
            d["Q"] = q
        elif "Q" in comp.state_dict():
            d["Q"] = comp.state_dict()["Q"]
        comp.load_state_dict(d)
