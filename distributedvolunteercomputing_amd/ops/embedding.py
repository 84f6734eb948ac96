"""Token (+ learned position) embedding: HIP gather forward, fp32-atomic scatter backward.

Graph-capture safe (fixed launch shapes, no data-dependent sizes), unlike torch's
sort/segment embedding backward, and the position add of GPT-2 is fused into the gather.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import native, use_native


class _Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe, T):
        idx = idx.contiguous()
        ctx.save_for_backward(idx)
        ctx.V, ctx.T = wte.shape[0], T
        ctx.Tpos = 0 if wpe is None else wpe.shape[0]
        return native().embed_fwd(idx, wte, wpe, T)

    @staticmethod
    def backward(ctx, dx):
        (idx,) = ctx.saved_tensors
        dwte, dwpe = native().embed_bwd(idx, dx.contiguous(), ctx.V, ctx.T, ctx.Tpos)
        return None, dwte, dwpe, None


def embed(idx: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor | None = None) -> torch.Tensor:
    """idx [B, T] -> [B, T, C] = wte[idx] (+ wpe[:T])."""
    B, T = idx.shape
    if use_native(wte) and wte.dtype == torch.bfloat16:
        return _Embed.apply(idx, wte, wpe, T).view(B, T, -1)
    x = F.embedding(idx, wte)
    if wpe is not None:
        x = x + wpe[:T]
    return x
