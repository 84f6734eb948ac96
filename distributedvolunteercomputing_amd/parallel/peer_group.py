"""A group of volunteer peers that can be rebuilt on membership change.

Each generation of the training membership gets its OWN raw c10d process group, created
directly from a (prefixed) store with ``ProcessGroupNCCL`` (RCCL on ROCm, over xGMI) or
``ProcessGroupGloo`` (CPU volunteers / tests). Unlike ``dist.new_group`` this does not need
every member of the *previous* generation to take part, so survivors can re-form a group
after a peer has died (SURVEY.md §5.3 "(N) dropout-tolerant averaging").

Reference analog: the coordinator's ``clients`` pool mutated by join/end verbs
(/root/reference/server.py:104-154) — here the pool is a generation-numbered member list.
"""
from __future__ import annotations

import datetime as _dt
import os

import torch
import torch.distributed as dist


def _gloo_pg(store, rank, size, timeout):
    opts = dist.ProcessGroupGloo._Options()
    opts._timeout = timeout
    host = os.environ.get("VCX_GLOO_HOST", "127.0.0.1")
    opts._devices = [dist.ProcessGroupGloo.create_device(hostname=host)]
    return dist.ProcessGroupGloo(store, rank, size, opts)


def _nccl_pg(store, rank, size, timeout):
    return dist.ProcessGroupNCCL(store, rank, size, timeout)


class PeerGroup:
    """One generation of live peers: rank/size are positions in ``members``."""

    def __init__(self, store, rank: int, size: int, backend: str = "gloo", *, generation: int = 0,
                 members=None, timeout_s: float = 300.0, device=None):
        self.generation = generation
        self.members = list(members) if members is not None else list(range(size))
        self.rank = rank
        self.size = size
        self.backend = backend
        self.device = device
        timeout = _dt.timedelta(seconds=timeout_s)
        prefixed = dist.PrefixStore(f"vcx/pg/{generation}", store)
        if size == 1:
            self.pg = None
        elif backend == "nccl":
            self.pg = _nccl_pg(prefixed, rank, size, timeout)
        elif backend == "gloo":
            self.pg = _gloo_pg(prefixed, rank, size, timeout)
        else:
            raise ValueError(f"unknown backend {backend!r}")

    @classmethod
    def from_default(cls, device=None) -> "PeerGroup":
        """Wrap torch.distributed's default process group (e.g. the torchrun world)."""
        self = cls.__new__(cls)
        self.generation = 0
        self.size = dist.get_world_size()
        self.rank = dist.get_rank()
        self.members = list(range(self.size))
        self.backend = dist.get_backend()
        self.device = device
        self.pg = dist.distributed_c10d._get_default_group() if self.size > 1 else None
        return self

    # ------------------------------------------------------------------ collectives
    def allreduce_(self, t: torch.Tensor):
        if self.pg is None:
            return t
        self.pg.allreduce([t]).wait()
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0):
        if self.pg is None:
            return t
        opts = dist.BroadcastOptions()
        opts.rootRank = root
        opts.rootTensor = 0
        self.pg.broadcast([t], opts).wait()
        return t

    def reduce_scatter_(self, out: torch.Tensor, inp: torch.Tensor):
        """out (numel = inp.numel()/size) <- sum over peers of this peer's slice of inp."""
        if self.pg is None:
            out.copy_(inp)
            return out
        if self.backend == "gloo":  # gloo lacks reduce_scatter_base: all-reduce then slice
            tmp = inp.clone()
            self.pg.allreduce([tmp]).wait()
            n = out.numel()
            out.copy_(tmp[self.rank * n : (self.rank + 1) * n])
            return out
        self.pg._reduce_scatter_base(out, inp).wait()
        return out

    def all_gather_(self, out: torch.Tensor, inp: torch.Tensor):
        if self.pg is None:
            out.copy_(inp)
            return out
        self.pg._allgather_base(out, inp).wait()
        return out

    def all_gather_object_sizes(self, n: int):
        """All-gather one int per peer (small metadata exchange)."""
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.tensor([n], dtype=torch.int64, device=dev)
        out = torch.zeros(self.size, dtype=torch.int64, device=dev)
        if self.pg is None:
            return [n]
        self.pg._allgather_base(out, t).wait()
        return out.tolist()

    def send(self, t: torch.Tensor, dst: int, tag: int = 0):
        self.pg.send([t], dst, tag).wait()

    def recv(self, t: torch.Tensor, src: int, tag: int = 0):
        self.pg.recv([t], src, tag).wait()

    def exchange(self, send_t: torch.Tensor, recv_t: torch.Tensor, peer: int, tag: int = 0):
        """Pairwise swap with `peer`. The lower rank sends first, the higher receives first,
        which keeps blocking RCCL/gloo point-to-point deadlock-free without group calls."""
        if self.rank < peer:
            self.send(send_t, peer, tag)
            self.recv(recv_t, peer, tag)
        else:
            self.recv(recv_t, peer, tag)
            self.send(send_t, peer, tag)

    def exchange_all(self, send_t: torch.Tensor, recv_t: torch.Tensor, send_to: int, recv_from: int | None = None):
        """One round in which EVERY rank of the group sends `send_t` to `send_to` and receives
        `recv_t` from `recv_from` (default: the same peer). Issued as ONE alltoall whose only
        non-empty splits are those two, so RCCL runs it as grouped send/recv: both directions of
        the xGMI link at once (the blocking `exchange` above serialises them)."""
        recv_from = send_to if recv_from is None else recv_from
        ins = [0] * self.size
        outs = [0] * self.size
        ins[send_to] = send_t.numel()
        outs[recv_from] = recv_t.numel()
        self.pg.alltoall_base(recv_t.view(-1), send_t.view(-1), outs, ins, dist.AllToAllOptions()).wait()

    def barrier(self):
        if self.pg is None:
            return
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.zeros(1, device=dev)
        self.pg.allreduce([t]).wait()
        if self.backend == "nccl":
            torch.cuda.synchronize()

    def shutdown(self):
        pg, self.pg = self.pg, None
        if pg is not None and self.backend == "nccl":
            try:
                pg.shutdown()
            except Exception:
                pass
