"""Causal self-attention on a packed QKV tensor [B, T, 3, H, D] -> [B, T, H, D].

GPU, D == 64: the hand-written MFMA flash-attention kernels of ``attention.hip`` (forward,
dK/dV and dQ backward) that read the packed projection output and write the packed gradient
directly, so no permute/contiguous/cat kernels surround attention. Other head dims and CPU
tensors use torch SDPA on unpacked views (the reference path / numerics oracle).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ._lib import native, use_native


class _Attn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, scale):
        C = native()
        out, lse = C.attn_fwd(qkv, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        return native().attn_bwd(qkv, out, dout.contiguous(), lse, ctx.scale), None


def _ref(qkv, scale):
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale)
    return y.transpose(1, 2)


def causal_attention(qkv: torch.Tensor, scale: float | None = None) -> torch.Tensor:
    """qkv [B, T, 3, H, D] -> out [B, T, H, D] (causal)."""
    D = qkv.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if use_native(qkv) and D == 64 and qkv.dtype == torch.bfloat16:
        return _Attn.apply(qkv.contiguous(), scale)
    return _ref(qkv, scale)
