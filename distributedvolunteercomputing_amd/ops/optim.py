"""Flat-buffer optimizer and local-SGD kernels (HIP on GPU, torch reference on CPU).

`ostate` is a 4-float device tensor {step, lr, clip_coef, grad_sumsq}; see optim.hip.
"""
from __future__ import annotations

import torch

from ._lib import native, use_native

OS_STEP, OS_LR, OS_CLIP, OS_SUMSQ = 0, 1, 2, 3


def new_ostate(device, lr: float) -> torch.Tensor:
    s = torch.zeros(4, dtype=torch.float32, device=device)
    s[OS_LR] = lr
    s[OS_CLIP] = 1.0
    return s


def adamw_step(param, grad, master, m, v, ostate, *, n_decay, beta1, beta2, eps, wd, max_norm=0.0):
    """One AdamW step on flat buffers (graph-capturable on GPU)."""
    if use_native(param):
        C = native()
        if max_norm > 0:
            ostate[OS_SUMSQ].zero_()
            C.grad_sumsq(grad, ostate)
        C.adam_prologue(ostate, float(max_norm))
        C.adamw_flat(param, grad, master, m, v, int(n_decay), ostate, beta1, beta2, eps, wd)
        return
    # ---- CPU reference (same math, fp32)
    g = grad.float()
    ostate[OS_STEP] += 1
    coef = 1.0
    if max_norm > 0:
        nrm = g.norm().item()
        coef = min(1.0, max_norm / (nrm + 1e-6))
        ostate[OS_SUMSQ] = nrm * nrm
    ostate[OS_CLIP] = coef
    step = ostate[OS_STEP].item()
    lr = ostate[OS_LR].item()
    g = g * coef
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    denom = v.sqrt() / (bc2**0.5) + eps
    if n_decay > 0:
        master[:n_decay].mul_(1 - lr * wd)
    master.addcdiv_(m, denom, value=-lr / bc1)
    param.copy_(master.to(param.dtype))


def lsgd_delta(master, anchor, delta):
    if use_native(master) and delta.dtype == torch.bfloat16:
        native().lsgd_delta(master, anchor, delta)
    else:
        delta.copy_((master - anchor).to(delta.dtype))


def lsgd_apply(avg, anchor, master, param, mom=None, *, outer_lr=1.0, mu=0.0, nesterov=False, avg_scale=1.0):
    if use_native(avg) and avg.dtype == torch.bfloat16:
        native().lsgd_apply(avg, anchor, master, param, mom, outer_lr, mu, nesterov, avg_scale)
        return
    g = -avg.float() * avg_scale
    upd = g
    if mom is not None:
        mom.mul_(mu).add_(g)
        upd = g + mu * mom if nesterov else mom
    anchor.add_(upd, alpha=-outer_lr)
    master.copy_(anchor)
    param.copy_(anchor.to(param.dtype))


def f32_to_bf16(src, dst):
    if use_native(src):
        native().f32_to_bf16(src, dst)
    else:
        dst.copy_(src.to(dst.dtype))


def axpy_bf16(src, acc, scale=1.0):
    """acc += scale * src (bf16 buffers)."""
    if use_native(src):
        native().axpy_bf16(src, acc, scale)
    else:
        acc.copy_((acc.float() + scale * src.float()).to(acc.dtype))


def reduce_bcast_bf16(inp, out, mine, P: int):
    """Direct all-reduce middle step: sum the P rows of `inp`; write the sum to every row of
    `out` (may alias `inp`: each element is read before it is written) and to `mine`."""
    if use_native(inp):
        native().reduce_bcast_bf16(inp, out, mine, P)
        return
    red = inp.view(P, -1).float().sum(0).to(inp.dtype)
    if out is not None:
        out.view(P, -1).copy_(red.unsqueeze(0).expand(P, -1))
    if mine is not None:
        mine.copy_(red)
