"""Flat parameter / gradient storage.

Every parameter of a module is re-homed into ONE contiguous buffer (and its gradient into a
second one) so that the optimizer, the local-SGD averaging, compression and optimizer-state
sharding each operate on a single 1-D tensor: one kernel launch for AdamW, one collective per
bucket, trivial sharding (contiguous slices) and trivial re-sharding when peers join/leave.

Layout: [decayed params (dim >= 2) | non-decayed params (biases, norm gains)], each segment
aligned to ``ALIGN`` elements (128 B for bf16) so vectorised 16-B accesses never straddle.
A 4-D parameter that is channels-last (a ResNet convolution after ``.to(memory_format=
torch.channels_last)``) keeps that layout in its segment: its parameter and gradient views have
channels-last strides, so the NHWC convolution kernels take the weight and return its gradient
without a layout copy each way (ResNet-50: ~48 copies per step, profiles/r4_resnet50_ab.txt).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

ALIGN = 64
# total length is padded to a multiple of ALIGN * lcm(1..8) so that the flat space splits into
# equal, 128-B-aligned shards for ANY peer count 1..8 (elastic re-sharding never re-pads)
SHARD_PAD = ALIGN * 840


def _round_up(n, a=ALIGN):
    return (n + a - 1) // a * a


@dataclass
class Segment:
    name: str
    offset: int
    numel: int
    shape: tuple
    decay: bool
    channels_last: bool = False


def _channels_last(p: torch.Tensor) -> bool:
    """4-D and stored channels-last (and not also plain-contiguous, as 1x1 kernels are both)."""
    return p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous()


def segment_view(buf: torch.Tensor, s: Segment) -> torch.Tensor:
    """Segment `s` of a flat buffer as a tensor of its parameter's shape (and memory format)."""
    v = buf[s.offset : s.offset + s.numel]
    if s.channels_last:
        n, c, h, w = s.shape
        return v.view(n, h, w, c).permute(0, 3, 1, 2)
    return v.view(s.shape)


class FlatParams:
    def __init__(self, module: torch.nn.Module, dtype=torch.bfloat16, device=None, pad_to: int = SHARD_PAD):
        params = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        seen = {}
        uniq = []
        for n, p in params:  # tied weights appear once
            if id(p) in seen:
                continue
            seen[id(p)] = n
            uniq.append((n, p))
        decay = [(n, p) for n, p in uniq if p.dim() >= 2]
        nodecay = [(n, p) for n, p in uniq if p.dim() < 2]
        device = device or (uniq[0][1].device if uniq else torch.device("cpu"))
        self.segments: list[Segment] = []
        off = 0
        for group, is_decay in ((decay, True), (nodecay, False)):
            for n, p in group:
                self.segments.append(Segment(n, off, p.numel(), tuple(p.shape), is_decay, _channels_last(p)))
                off = _round_up(off + p.numel())
            if is_decay:
                self.n_decay = off
        self.numel = _round_up(max(off, pad_to), pad_to)
        self.dtype = dtype
        self.param = torch.zeros(self.numel, dtype=dtype, device=device)
        self.grad = torch.zeros(self.numel, dtype=dtype, device=device)
        self._params = []
        byname = dict(uniq)
        with torch.no_grad():
            for s in self.segments:
                p = byname[s.name]
                view = segment_view(self.param, s)
                view.copy_(p.detach().to(device=device, dtype=dtype))
                p.data = view
                p.grad = segment_view(self.grad, s)
                self._params.append(p)

    def zero_grad(self):
        self.grad.zero_()

    def rebind_grads(self):
        """Re-point .grad at the flat buffer (call if something replaced p.grad)."""
        for s, p in zip(self.segments, self._params):
            p.grad = segment_view(self.grad, s)

    def state_dict_views(self, flat: torch.Tensor):
        """Name -> view of an arbitrary flat buffer with this layout (for checkpoints)."""
        return {s.name: segment_view(flat, s) for s in self.segments}

    def shard_bounds(self, rank: int, world: int, align: int = ALIGN):
        """Contiguous [lo, hi) slice of the flat space owned by `rank` (ZeRO-style). For world
        sizes dividing 840 all shards have the same, aligned length."""
        if (self.numel // align) % world == 0:
            per = self.numel // world
        else:
            per = _round_up((self.numel + world - 1) // world, align)
        lo = min(rank * per, self.numel)
        hi = min(lo + per, self.numel)
        return lo, hi


class FlatBuffers:
    """Floating-point module buffers (BatchNorm running mean/var) gathered into one flat fp32
    vector, so the trainers average them with ONE small collective per synchronisation, hand
    them to newcomers and store them in checkpoints (BASELINE.json config 3, ResNet-50).
    Integer buffers (``num_batches_tracked``) are left alone."""

    def __init__(self, module: torch.nn.Module):
        self.entries = []  # (owner module, buffer name, qualified name, numel, shape)
        for qn, b in module.named_buffers():
            if b is None or not b.dtype.is_floating_point:
                continue
            mod_name, _, bname = qn.rpartition(".")
            owner = module.get_submodule(mod_name) if mod_name else module
            self.entries.append((owner, bname, qn, b.numel(), tuple(b.shape)))
        self.numel = sum(e[3] for e in self.entries)

    def __bool__(self):
        return self.numel > 0

    def as_fp32(self) -> torch.Tensor:
        """All buffers in one fp32 vector (a copy), in entry order."""
        if not self.entries:
            return torch.zeros(0)
        return torch.cat([owner._buffers[bn].detach().float().reshape(-1) for owner, bn, *_ in self.entries])

    def load_fp32(self, vec: torch.Tensor):
        pos = 0
        for owner, bn, qn, n, shape in self.entries:
            b = owner._buffers[bn]
            b.copy_(vec[pos : pos + n].view(shape).to(device=b.device, dtype=b.dtype))
            pos += n

    def names(self):
        return [qn for _, _, qn, *_ in self.entries]

    def averaged(self, group):
        """The mean over the group's peers as a new fp32 vector (None when there is nothing to
        average). The live buffers are not touched: an elastic round loads the result only after
        its verdict is `commit`, so an aborted round leaves every peer's buffers as they were."""
        if not self.entries or group is None or group.size == 1:
            return None
        v = self.as_fp32()
        dev = group.device if group.backend == "nccl" else "cpu"
        v = v.to(dev)
        group.allreduce_(v)
        return v.div_(group.size)

    def average_(self, group):
        """Mean over the group's peers, loaded into the live buffers (non-elastic callers)."""
        v = self.averaged(group)
        if v is not None:
            self.load_fp32(v)
