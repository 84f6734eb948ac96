"""Token (+ learned position) embedding: HIP gather forward; backward = fp32-atomic scatter for the
token table and a batch reduction for the position table, added into the flat .grad buffers.

Graph-capture safe (fixed launch shapes, no data-dependent sizes), unlike torch's
sort/segment embedding backward, and the position add of GPT-2 is fused into the gather.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import grad_buffer, native, use_native


class _Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe, T):
        idx = idx.contiguous()
        ctx.save_for_backward(idx)
        ctx.tables = (wte, wpe)
        ctx.V, ctx.T = wte.shape[0], T
        ctx.Tpos = 0 if wpe is None else wpe.shape[0]
        return native().embed_fwd(idx, wte, wpe, T)

    @staticmethod
    def backward(ctx, dx):
        (idx,) = ctx.saved_tensors
        wte, wpe = ctx.tables
        ctx.tables = None
        gte, gpe = grad_buffer(wte), grad_buffer(wpe)
        dwte, dwpe = native().embed_bwd(idx, dx.contiguous(), ctx.V, ctx.T, ctx.Tpos, gte, gpe)
        # gradients added into preset (flat) .grad buffers are not handed to autograd again
        return None, (None if gte is not None else dwte), (None if gpe is not None or ctx.Tpos == 0 else dwpe), None


def embed(idx: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor | None = None) -> torch.Tensor:
    """idx [B, T] -> [B, T, C] = wte[idx] (+ wpe[:T])."""
    B, T = idx.shape
    if use_native(wte) and wte.dtype == torch.bfloat16:
        return _Embed.apply(idx, wte, wpe, T).view(B, T, -1)
    x = F.embedding(idx, wte)
    if wpe is not None:
        x = x + wpe[:T]
    return x
