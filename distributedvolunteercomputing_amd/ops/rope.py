"""Rotary position embedding fused with the QKV split (Llama-3 attention).

``rope_qkv(qkv, cos, sin, Hq, Hkv)``: qkv [B, T, (Hq + 2 Hkv) * D] -> q [B, Hq, T, D],
k [B, Hkv, T, D] (both rotated on interleaved pairs, the convention of the Llama reference
code) and v [B, Hkv, T, D]. GPU: one HIP kernel each way (csrc/kernels/rope.hip); CPU: torch.
"""
from __future__ import annotations

import torch

from ._lib import native, use_native


def rope_tables(T: int, hd: int, theta: float, device):
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, device=device, dtype=torch.float32) / hd))
    f = torch.outer(torch.arange(T, device=device, dtype=torch.float32), inv)
    return f.cos().contiguous(), f.sin().contiguous()


def apply_rope(x, cos, sin):
    """x [B, H, T, hd]: rotate interleaved pairs (reference path)."""
    x2 = x.float().unflatten(-1, (-1, 2))
    a, b = x2[..., 0], x2[..., 1]
    c, s = cos[None, None, : x.shape[2]], sin[None, None, : x.shape[2]]
    return torch.stack([a * c - b * s, a * s + b * c], -1).flatten(-2).to(x.dtype)


class _RopeQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, Hq, Hkv):
        ctx.save_for_backward(cos, sin)
        return tuple(native().rope_qkv_fwd(qkv.contiguous(), cos, sin, Hq, Hkv))

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        dqkv = native().rope_qkv_bwd(dq.contiguous(), dk.contiguous(), dv.contiguous(), cos, sin)
        return dqkv, None, None, None, None


def rope_qkv(qkv, cos, sin, Hq: int, Hkv: int):
    B, T, W = qkv.shape
    hd = W // (Hq + 2 * Hkv)
    if use_native(qkv) and qkv.dtype == torch.bfloat16 and hd % 8 == 0:
        return _RopeQKV.apply(qkv, cos, sin, Hq, Hkv)
    q, k, v = qkv.split([Hq * hd, Hkv * hd, Hkv * hd], -1)
    q = apply_rope(q.reshape(B, T, Hq, hd).transpose(1, 2), cos, sin)
    k = apply_rope(k.reshape(B, T, Hkv, hd).transpose(1, 2), cos, sin)
    return q, k, v.reshape(B, T, Hkv, hd).transpose(1, 2)
