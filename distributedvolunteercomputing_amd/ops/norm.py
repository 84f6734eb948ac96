"""LayerNorm / RMSNorm with an optional fused residual add (HIP on GPU, torch on CPU).

``add_layernorm(a, b, w, bias, branch_bias=bb)`` returns ``(y, x)`` with ``x = a + b + bb``
(the new residual stream) and ``y = LN(x)``. Fusing the add saves one full read+write of the
residual stream per sub-layer; ``bb`` is the bias of the GEMM that produced ``b`` (the GEMM
then runs without a bias epilogue and its bias gradient comes out of this kernel's backward
as the column sums of dx, replacing a separate reduction). The backward also fuses the
residual-gradient add into ``dx``.
"""
from __future__ import annotations

import torch

from ._lib import grad_buffer, native, use_native


def _ref_ln(x, w, b, eps, rms):
    xf = x.float()
    if rms:
        var = xf.pow(2).mean(-1, keepdim=True)
        y = xf * torch.rsqrt(var + eps)
    else:
        mu = xf.mean(-1, keepdim=True)
        var = (xf - mu).pow(2).mean(-1, keepdim=True)
        y = (xf - mu) * torch.rsqrt(var + eps)
    y = y * w.float()
    if b is not None:
        y = y + b.float()
    return y.to(x.dtype)


class _AddLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, w, bias, eps, rms, bb):
        C = native()
        y, x, mean, rstd = C.ln_fwd(a.contiguous(), None if b is None else b.contiguous(), w, bias, eps, rms, bb)
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.params = (w, bias, bb)  # for their preset .grad buffers (not saved tensors: never modified)
        ctx.has_b = b is not None
        ctx.has_bias = bias is not None
        ctx.has_bb = bb is not None
        ctx.rms = rms
        # an unused residual output (the last block's) gets no zero-filled gradient: dx_res None -> no residual add
        ctx.set_materialize_grads(False)
        if b is None:
            x = x.view_as(x)  # output aliases the input: hand autograd a view, not the input itself
        return y, x

    @staticmethod
    def backward(ctx, dy, dx_res):
        if dy is None:  # only the residual output was used: it is a + b (+ bb)
            if dx_res is None:
                return None, None, None, None, None, None, None
            dbb = None
            if ctx.has_bb:
                dbb = dx_res.reshape(-1, dx_res.shape[-1]).float().sum(0).to(dx_res.dtype)
            return dx_res, (dx_res if ctx.has_b else None), None, None, None, None, dbb
        x, w, mean, rstd = ctx.saved_tensors
        C = native()
        dres = None if dx_res is None else dx_res.contiguous()
        pw, pbias, pbb = ctx.params
        gw, gb, gbb = grad_buffer(pw), grad_buffer(pbias) if ctx.has_bias else None, grad_buffer(pbb) if ctx.has_bb else None
        dx, dw, dbias, dbb = C.ln_bwd(dy.contiguous(), x, w, mean, rstd, dres, ctx.has_bias, ctx.rms, ctx.has_bb,
                                      gw, gb, gbb)
        # parameter gradients already added into preset buffers are not handed to autograd again
        dw = None if gw is not None else dw
        dbias = None if gb is not None else dbias
        dbb = None if gbb is not None else dbb
        return dx, (dx if ctx.has_b else None), dw, dbias, None, None, dbb


def add_layernorm(a, b, weight, bias=None, eps: float = 1e-5, rms: bool = False, branch_bias=None):
    """Returns (LN(a+b[+branch_bias]), a+b[+branch_bias]). With b=None returns (LN(a), a)."""
    if use_native(a):
        y, x = _AddLN.apply(a, b, weight, bias, eps, rms, branch_bias)
        return y, x
    if b is None:
        x = a
    else:
        x = a + (b if branch_bias is None else b + branch_bias)
    return _ref_ln(x, weight, bias, eps, rms), x


def layernorm(x, weight, bias=None, eps: float = 1e-5):
    return add_layernorm(x, None, weight, bias, eps, False)[0]


def rmsnorm(x, weight, eps: float = 1e-6):
    return add_layernorm(x, None, weight, None, eps, True)[0]


def add_rmsnorm(a, b, weight, eps: float = 1e-6):
    return add_layernorm(a, b, weight, None, eps, True)
