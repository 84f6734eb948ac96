"""Linear layer whose backward computes the weight gradient as a split-M batched GEMM.

The weight gradient of a token-major linear layer, dW[N, K] = dY[M, N]^T X[M, K], reduces over
all M = B*T tokens (65536 at the GPT-2 bench shape) into a small output: a single library GEMM
has only (N/256)*(K/256) output tiles (9..36 at GPT-2-small sizes) for 256 CUs and runs at
0.33-0.77 PF/s. Splitting the token axis into S chunks and issuing ONE batched GEMM
(S x more tiles in flight) measured 1.3-2.3x faster on MI355X (scripts/gemm_probe.py,
PROBE_SPLITS: qkv 399 -> 243 us, proj 234 -> 100 us, fc 401 -> 301 us, fc2 413 -> 309 us).
The S partial products are summed in fp32 by a HIP kernel directly INTO the flat gradient
buffer (``p.grad`` is a view of it, see parallel/flat_params.py), so no separate autograd
accumulation pass runs either.

Forward, input gradient and bias gradient are library GEMMs / reductions (hipBLASLt / rocBLAS
through the TunableOp table, utils/tuning.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import grad_buffer, native, use_native

MIN_ROWS_PER_SPLIT = 2048


def _splits(M: int, N: int, K: int) -> int:
    if N * K >= 16 * 1024 * 1024:  # big outputs (LM head) already fill the GPU
        s = 4
    else:
        s = 16
    while s > 1 and (M % s or M // s < MIN_ROWS_PER_SPLIT):
        s //= 2
    return s


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False):
    """dW = dy2^T @ x2 ([M, N], [M, K] -> [N, K]); written into / added onto `out` if given."""
    M, N = dy2.shape
    K = x2.shape[1]
    S = _splits(M, N, K)
    if S == 1 or not use_native(dy2) or (N * K) % 8:
        g = dy2.t().mm(x2)
        if out is None:
            return g
        if accumulate:
            out.add_(g)
        else:
            out.copy_(g)
        return out
    part = torch.bmm(dy2.view(S, M // S, N).transpose(1, 2), x2.view(S, M // S, K))  # [S, N, K]
    if out is None:
        out = torch.empty(N, K, device=dy2.device, dtype=dy2.dtype)
        accumulate = False
    native().splitk_reduce(part, out, accumulate)
    return out


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.bias = b
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, K = w.shape
        dy2 = dy.reshape(-1, N)
        x2 = x.reshape(-1, K)
        dx = dy2.mm(w).view(x.shape) if ctx.needs_input_grad[0] else None
        dw = db = None
        if ctx.needs_input_grad[1]:
            g = w.grad
            if g is not None and g.is_contiguous() and g.dtype == w.dtype and g.shape == w.shape:
                wgrad(dy2, x2, out=g, accumulate=True)  # straight into the (flat) .grad; autograd adds nothing
            else:
                dw = wgrad(dy2, x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = grad_buffer(ctx.bias)
            if gb is not None and (N % 8) == 0:
                native().colsum_bf16(dy2.contiguous(), gb)  # HIP column sums added into the flat .grad
            elif (N % 8) == 0:
                db = native().colsum_bf16(dy2.contiguous())
            else:
                db = dy2.sum(0, dtype=torch.float32).to(dy.dtype)
        ctx.bias = None
        return dx, dw, db


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """y = x @ w^T (+ b), x [..., K], w [N, K]."""
    if use_native(w) and w.dtype == torch.bfloat16 and torch.is_grad_enabled() and w.requires_grad:
        return _Linear.apply(x, w, b)
    return F.linear(x, w, b)
