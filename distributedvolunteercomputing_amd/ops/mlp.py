"""GPT-2 MLP block ``fc2(gelu(fc(h) + b))`` with the GELU fused into hipBLASLt GEMM epilogues.

Forward: ONE hipBLASLt GEMM with the GELU_AUX_BIAS epilogue writes both gelu(h W1^T + b) (the fc2
input) and the pre-activation (kept for the backward), instead of a GEMM followed by a HIP
bias+GELU pass over the [tokens, 4C] activation. Backward: the fc2 input-gradient GEMM runs with
the DGELU_BGRAD epilogue, which multiplies by gelu'(pre-activation) and reduces the fc bias
gradient in the same kernel (no bias+GELU backward pass, no column-sum launches). Weight
gradients are the split-M batched GEMMs of ops/linear.py, added straight into the flat .grad.

If hipBLASLt offers no algorithm for an epilogue (checked once per process), the op falls back
to library GEMMs + the HIP bias_gelu kernels (ops/activations.py) — both native paths.
fc2's bias is not applied here: GPT-2 fuses it into the following residual-add + LayerNorm.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import activations
from ._lib import grad_buffer, native, use_native
from .linear import linear, wgrad

_LT = {"fwd": os.environ.get("VCX_LT_MLP", "1") != "0", "bwd": os.environ.get("VCX_LT_MLP", "1") != "0"}


def _wgrad_into(dy2, x2, p):
    g = grad_buffer(p)
    if g is not None:
        wgrad(dy2, x2, out=g, accumulate=True)
        return None
    return wgrad(dy2, x2)


class _GeluMLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, fc_w, fc_b, fc2_w):
        C = native()
        shp = h.shape
        h2 = h.reshape(-1, shp[-1]).contiguous()
        M, Fd = h2.shape[0], fc_w.shape[0]
        pre = torch.empty(M, Fd, device=h.device, dtype=h.dtype)
        act = torch.empty_like(pre)
        if not C.lt_matmul(h2, fc_w, act, False, True, C.LT_EPI_GELU_AUX_BIAS, fc_b, pre):
            raise RuntimeError("hipBLASLt GELU_AUX_BIAS epilogue unavailable")
        y = torch.mm(act, fc2_w.t())
        ctx.save_for_backward(h2, pre, act, fc_w, fc_b, fc2_w)
        ctx.fc_b = fc_b
        ctx.shape = shp
        return y.view(*shp[:-1], fc2_w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        C = native()
        h2, pre, act, fc_w, fc_b, fc2_w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        d_fc2 = _wgrad_into(dy2, act, fc2_w)
        gb = grad_buffer(ctx.fc_b)
        ctx.fc_b = None
        dpre = torch.empty_like(pre)
        db = torch.empty(pre.shape[1], device=pre.device, dtype=pre.dtype)
        if _LT["bwd"] and C.lt_matmul(dy2, fc2_w, dpre, False, False, C.LT_EPI_DGELU_BGRAD, db, pre):
            if gb is not None:
                gb.add_(db)
                db = None
        else:
            _LT["bwd"] = False
            # unfused: dact = dy W2, then the HIP GELU backward on the biased pre-activation
            dact = dy2.mm(fc2_w)
            dpre = native().gelu_bwd(pre, dact)
            if gb is not None:
                native().colsum_bf16(dpre, gb)
                db = None
            else:
                db = native().colsum_bf16(dpre)
        d_fc = _wgrad_into(dpre, h2, fc_w)
        dh = dpre.mm(fc_w).view(ctx.shape)
        return dh, d_fc, db, d_fc2


def gelu_mlp(h, fc_w, fc_b, fc2_w):
    """fc2(gelu_tanh(h fc_w^T + fc_b)) without fc2's bias."""
    if use_native(h) and h.dtype == torch.bfloat16 and torch.is_grad_enabled() and _LT["fwd"]:
        try:
            return _GeluMLP.apply(h, fc_w, fc_b, fc2_w)
        except RuntimeError as e:
            if "epilogue unavailable" not in str(e):
                raise
            _LT["fwd"] = False
    if use_native(h):
        return linear(activations.bias_gelu(linear(h, fc_w), fc_b), fc2_w)
    return F.linear(F.gelu((F.linear(h, fc_w) + fc_b).float(), approximate="tanh").to(h.dtype), fc2_w)
