"""All-reduce algorithms for averaging across volunteer peers.

* ``rccl``      — the library all-reduce of the peer group (RCCL over xGMI on MI355X: it runs
                  several rings/trees over the 7 point-to-point links at once). Default: the
                  averaging payload is one flat buffer, so a single large collective is the
                  per-link-bandwidth-optimal call.
* ``rs_ag``     — reduce-scatter + all-gather (the sharded form used by optimizer-state
                  sharding: each peer only needs its shard between the two halves).
* ``butterfly`` — recursive halving (reduce-scatter) + recursive doubling (all-gather) over
                  pairwise exchanges: log2(P) rounds, each with ONE partner, so every round is
                  one xGMI link at full rate and the schedule re-forms trivially over any live
                  set (non-power-of-two sets fold the extra peers in first).
* ``ring``      — classic 2(P-1)-step ring over pairwise exchanges.
* ``direct``    — one-shot reduce-scatter + all-gather over the full xGMI mesh: ONE all-to-all
                  in which every peer sends shard j of its buffer to peer j (P-1 links at once),
                  a fused HIP reduce that sums the P received copies of its own shard and writes
                  the sum once per destination, and ONE all-to-all that returns the reduced
                  shards. Each peer moves 2(P-1)/P of the buffer, spread over its P-1 = 7 links
                  concurrently: ~2·(S/8)/153 GB/s ≈ 0.4 ms for GPT-2-small's 248 MB of bf16
                  pseudo-gradient, against ~2.8 ms for a single ring on one link.
                  Works for any P (no power-of-two folding).

The reductions of the hand-written algorithms run in a HIP kernel (``axpy_bf16``) for bf16
GPU buffers. All functions SUM in place; the caller applies the 1/P scale (fused into the
local-SGD apply kernel).

No reference analog: the reference has no collectives.
"""
from __future__ import annotations

import torch

from .. import ops
from .peer_group import PeerGroup

ALGOS = ("rccl", "rs_ag", "butterfly", "ring", "direct")


def _add_(acc: torch.Tensor, src: torch.Tensor):
    if acc.dtype == torch.bfloat16 and acc.is_cuda and acc.numel() % 8 == 0:
        ops.axpy_bf16(src, acc, 1.0)
    else:
        acc.add_(src)


def allreduce_sum_(t: torch.Tensor, group: PeerGroup, algo: str = "rccl") -> torch.Tensor:
    if group is None or group.size == 1:
        return t
    if algo == "rccl":
        return group.allreduce_(t)
    if algo == "rs_ag":
        return _rs_ag(t, group)
    if algo == "butterfly":
        return _butterfly(t, group)
    if algo == "ring":
        return _ring(t, group)
    if algo == "direct":
        return _direct(t, group)
    raise ValueError(f"unknown all-reduce algorithm {algo!r}; choose from {ALGOS}")


def _pad_len(n: int, parts: int, align: int = 64) -> int:
    q = parts * align
    return (n + q - 1) // q * q


def _padded(t, L):
    """t itself when it already has length L (flat buffers are padded for P | 840), else a
    zero-padded copy."""
    n = t.numel()
    if L == n:
        return t
    buf = t.new_zeros(L)
    buf[:n].copy_(t)
    return buf


def _rs_ag(t, group):
    P = group.size
    n = t.numel()
    L = _pad_len(n, P)
    buf = _padded(t, L)
    shard = buf.new_empty(L // P)
    group.reduce_scatter_(shard, buf)
    group.all_gather_(buf, shard)
    if buf is not t:
        t.copy_(buf[:n])
    return t


def _swap(group, send_t, recv_t, peer, tag, all_ranks: bool):
    """Pairwise swap of one butterfly round. When EVERY rank of the group takes part in the round
    (power-of-two groups) it is one full-duplex alltoall (grouped send/recv); otherwise (folded
    peers are waiting outside the round) ordered blocking point-to-point."""
    if all_ranks:
        group.exchange_all(send_t, recv_t, peer)
    else:
        group.exchange(send_t, recv_t, peer, tag=tag)


def _butterfly(t, group):
    P, r = group.size, group.rank
    p2 = 1
    while p2 * 2 <= P:
        p2 *= 2
    n = t.numel()
    # --- fold: peers >= p2 hand their whole buffer to (rank - p2) and wait for the result
    extra = P - p2
    if r >= p2:
        group.send(t, r - p2, tag=1)
        group.recv(t, r - p2, tag=2)
        return t
    if r < extra:
        tmp = torch.empty_like(t)
        group.recv(tmp, r + p2, tag=1)
        _add_(t, tmp)
    # --- recursive halving reduce-scatter among the p2 core peers
    L = _pad_len(n, p2)
    buf = _padded(t, L)
    lo, hi = 0, L
    dist_ = p2 // 2
    segs = []
    while dist_ >= 1:
        peer = r ^ dist_
        mid = (lo + hi) // 2
        if r & dist_:  # keep upper half
            keep, give = (mid, hi), (lo, mid)
        else:
            keep, give = (lo, mid), (mid, hi)
        recv = buf.new_empty(keep[1] - keep[0])
        _swap(group, buf[give[0] : give[1]].contiguous(), recv, peer, 3, extra == 0)
        kv = buf[keep[0] : keep[1]]
        _add_(kv, recv)
        segs.append((lo, hi, dist_))
        lo, hi = keep
        dist_ //= 2
    # --- recursive doubling all-gather (reverse order)
    for plo, phi, d in reversed(segs):
        peer = r ^ d
        mid = (plo + phi) // 2
        mine = (lo, hi)
        other = (mid, phi) if mine[0] == plo else (plo, mid)
        recv = buf.new_empty(other[1] - other[0])
        _swap(group, buf[mine[0] : mine[1]].contiguous(), recv, peer, 4, extra == 0)
        buf[other[0] : other[1]].copy_(recv)
        lo, hi = plo, phi
    if buf is not t:
        t.copy_(buf[:n])
    # --- unfold: return the result to the folded peers
    if r < extra:
        group.send(t, r + p2, tag=2)
    return t


def _ring(t, group):
    P, r = group.size, group.rank
    n = t.numel()
    L = _pad_len(n, P)
    buf = _padded(t, L)
    cs = L // P
    chunks = [buf[i * cs : (i + 1) * cs] for i in range(P)]
    right, left = (r + 1) % P, (r - 1) % P
    recv = buf.new_empty(cs)

    def step(send_t, recv_t, tag):
        if P > 2:  # every rank sends right and receives left in the same round: one grouped alltoall
            group.exchange_all(send_t, recv_t, right, left)
            return
        # even ranks send first, odd ranks receive first: deadlock-free for blocking p2p
        if r % 2 == 0:
            group.send(send_t, right, tag)
            group.recv(recv_t, left, tag)
        else:
            group.recv(recv_t, left, tag)
            group.send(send_t, right, tag)

    for s in range(P - 1):  # reduce-scatter
        si = (r - s) % P
        ri = (r - s - 1) % P
        step(chunks[si].contiguous(), recv, tag=10)
        _add_(chunks[ri], recv)
    for s in range(P - 1):  # all-gather
        si = (r + 1 - s) % P
        ri = (r - s) % P
        step(chunks[si].contiguous(), recv, tag=11)
        chunks[ri].copy_(recv)
    if buf is not t:
        t.copy_(buf[:n])
    return t


def _direct(t, group):
    P, r = group.size, group.rank
    n = t.numel()
    L = _pad_len(n, P, 8 if t.dtype == torch.bfloat16 else 1)
    buf = _padded(t, L)
    m = L // P
    split = [m] * P
    recv = torch.empty_like(buf)  # [P, m]: row j = peer j's copy of MY shard
    group.alltoall_(recv, buf, split, split)
    send = recv  # reused: row j = the reduced shard, sent back to peer j
    mine = buf[r * m : (r + 1) * m]
    if buf.is_cuda and buf.dtype == torch.bfloat16:
        ops.reduce_bcast_bf16(recv, send, mine, P)
    else:
        red = recv.view(P, m).sum(0, dtype=torch.float32 if buf.dtype != torch.float64 else None).to(buf.dtype)
        mine.copy_(red)
        send = red.unsqueeze(0).expand(P, m).contiguous().view(-1)
    group.alltoall_(buf, send, split, split)
    if buf is not t:
        t.copy_(buf[:n])
    return t
