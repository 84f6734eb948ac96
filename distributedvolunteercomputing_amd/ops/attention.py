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

from ._lib import grad_buffer, native, use_native


class _Attn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, scale, bias):
        C = native()
        out, lse = C.attn_fwd(qkv, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.scale = scale
        ctx.bias = bias  # not used by the forward: only its gradient is produced here
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        C = native()
        bias, ctx.bias = ctx.bias, None
        if bias is None or not ctx.needs_input_grad[2]:
            return C.attn_bwd(qkv, out, dout.contiguous(), lse, ctx.scale), None, None
        # the backward kernels also emit per-block column sums of dqkv = the gradient of the bias
        # the QKV projection added (linear(..., bias_grad_elsewhere=True)): no pass over dqkv
        gb = grad_buffer(bias)
        dqkv, db = C.attn_bwd_bias(qkv, out, dout.contiguous(), lse, ctx.scale, gb)
        return dqkv, None, (None if gb is not None else db.view_as(bias))


def _ref(qkv, scale):
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale)
    return y.transpose(1, 2)


def fused_bias_grad_ok(qkv: torch.Tensor) -> bool:
    """True when causal_attention(qkv, bias=...) computes the QKV-bias gradient in its kernels."""
    return use_native(qkv) and qkv.shape[-1] == 64 and qkv.dtype == torch.bfloat16


def causal_attention(qkv: torch.Tensor, scale: float | None = None, bias: torch.Tensor | None = None) -> torch.Tensor:
    """qkv [B, T, 3, H, D] -> out [B, T, H, D] (causal).

    bias: the [3*H*D] bias already added into qkv by the projection, whose gradient this op then
    returns (only valid with ``linear(..., bias_grad_elsewhere=True)`` and when
    ``fused_bias_grad_ok(qkv)``; otherwise leave it None)."""
    D = qkv.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if fused_bias_grad_ok(qkv):
        return _Attn.apply(qkv.contiguous(), scale, bias)
    assert bias is None, "bias gradient fusion needs the native hd64 bf16 attention path"
    return _ref(qkv, scale)


# ------------------------------------------------------------------ head-major GQA (Llama family)
class _AttnHM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale):
        out, lse = native().attn_hm_fwd(q, k, v, scale)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq, dk, dv = native().attn_hm_bwd(q, k, v, out, dout.contiguous(), lse, ctx.scale)
        return dq, dk, dv, None


_GQA_SDPA = [True]  # SDPA's enable_gqa (no repeat_interleave copies); falls back if unsupported


def _ref_gqa(q, k, v, scale):
    rep = q.shape[1] // k.shape[1]
    if rep > 1 and _GQA_SDPA[0]:
        try:
            return F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale, enable_gqa=True).transpose(1, 2)
        except (RuntimeError, TypeError):
            _GQA_SDPA[0] = False
    if rep > 1:
        k = k.repeat_interleave(rep, dim=1)
        v = v.repeat_interleave(rep, dim=1)
    return F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=scale).transpose(1, 2)


def gqa_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float | None = None) -> torch.Tensor:
    """Causal grouped-query attention, q [B, Hq, T, D], k / v [B, Hkv, T, D] (head-major, as
    ``rope_qkv`` returns them) -> out [B, T, Hq, D] (token-major: the output projection's input).
    GPU bf16 with D in (64, 128): the HIP kernels of attention_hm.hip; otherwise torch SDPA."""
    D = q.shape[-1]
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if use_native(q) and q.dtype == torch.bfloat16 and D in (64, 128) and q.shape[1] % k.shape[1] == 0:
        return _AttnHM.apply(q.contiguous(), k.contiguous(), v.contiguous(), scale)
    return _ref_gqa(q, k, v, scale)
