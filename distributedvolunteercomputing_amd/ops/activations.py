"""tanh-GELU (GPT-2 MLP) and SwiGLU (Llama MLP): HIP kernels on GPU, torch on CPU."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import grad_buffer, native, use_native


class _Gelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        ctx.save_for_backward(x)
        return native().gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return native().gelu_bwd(x, dy.contiguous())


def gelu(x):
    if use_native(x):
        return _Gelu.apply(x)
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b):
        x = x.contiguous()
        ctx.save_for_backward(x, b)
        ctx.bias = b
        return native().bias_gelu_fwd(x, b)

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        gb = grad_buffer(ctx.bias)
        ctx.bias = None
        dx, db = native().bias_gelu_bwd(x, b, dy.contiguous(), gb)
        return dx, (None if gb is not None else db)


def bias_gelu(x, b):
    """gelu_tanh(x + b) with the bias gradient reduced inside the backward kernel."""
    if use_native(x):
        return _BiasGelu.apply(x, b)
    return F.gelu((x + b).float(), approximate="tanh").to(x.dtype)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return native().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        return native().swiglu_bwd(gu, dy.contiguous())


def swiglu(gu):
    """gu = [..., 2F] laid out as [gate | up]; returns silu(gate) * up."""
    if use_native(gu):
        return _SwiGLU.apply(gu)
    g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)
