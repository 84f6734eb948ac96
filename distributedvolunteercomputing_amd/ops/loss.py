"""Fused softmax cross-entropy over a (possibly padded) vocabulary.

Rows that fit in registers (vocab <= 57344, e.g. GPT-2's 50304): ONE kernel per step reads
each logits row once, returns the row loss and overwrites the row IN PLACE with the gradient
(softmax - onehot) / n_valid (the logits are dead after the loss). The backward then only
rescales if the incoming gradient is not 1 (a device-side test, no host sync). 13.2 GB of HBM
traffic at the GPT-2 bench shape instead of 19.8 GB.

Larger vocabularies (Llama-3: 128256): forward = online max/sum per row (one read), backward =
in-place gradient scaled by a device-side scalar.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import config
from ._lib import native, use_native


class _XEntFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, vocab, ignore_index, nvalid, loss_rows):
        ctx.logits = logits  # holds the gradient now
        return loss_rows.sum() / nvalid

    @staticmethod
    def backward(ctx, dloss):
        d = ctx.logits
        ctx.logits = None
        native().xent_rescale(d, dloss.float().reshape(1).contiguous())
        return d, None, None, None, None, None


class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, vocab, ignore_index):
        C = native()
        loss_rows, lse = C.xent_fwd(logits, targets, vocab)
        valid = (targets != ignore_index) & (targets >= 0)
        nvalid = valid.sum().clamp_min(1).to(torch.float32)
        ctx.logits = logits  # not save_for_backward: the backward overwrites it in place
        ctx.save_for_backward(targets, lse, nvalid)
        ctx.vocab = vocab
        return loss_rows.sum() / nvalid

    @staticmethod
    def backward(ctx, dloss):
        targets, lse, nvalid = ctx.saved_tensors
        logits = ctx.logits
        ctx.logits = None
        gscale = (dloss.float() / nvalid).reshape(1).contiguous()
        native().xent_bwd(logits, targets, lse, gscale, logits, ctx.vocab)
        return logits, None, None, None


def cross_entropy(logits, targets, vocab: int | None = None, ignore_index: int = -100):
    """Mean cross-entropy. `logits` [N, Vp] (Vp >= vocab, padded columns ignored)."""
    vocab = vocab or logits.shape[-1]
    logits = logits.reshape(-1, logits.shape[-1])
    targets = targets.reshape(-1)
    if use_native(logits):
        logits, targets = logits.contiguous(), targets.contiguous().long()
        if logits.requires_grad and ignore_index < 0:  # the kernel treats target < 0 as ignored
            nvalid = ((targets != ignore_index) & (targets >= 0)).sum().clamp_min(1).to(torch.float32).reshape(1)
            with torch.no_grad():
                rows = native().xent_fused(logits.detach(), targets, nvalid, vocab)
            if rows is not None:
                return _XEntFused.apply(logits, targets, vocab, ignore_index, nvalid, rows)
        return _XEnt.apply(logits, targets, vocab, ignore_index)
    return F.cross_entropy(logits[:, :vocab].float(), targets.long(), ignore_index=ignore_index)


# ------------------------------------------------------------------ LM head + cross-entropy
_CHUNK_BUF: dict = {}


def _chunk_buf(rows: int, cols: int, dev) -> torch.Tensor:
    key = (rows, cols, dev)
    b = _CHUNK_BUF.get(key)
    if b is None:
        b = _CHUNK_BUF[key] = torch.empty(rows, cols, device=dev, dtype=torch.bfloat16)
    return b


class _LMHeadXEnt(torch.autograd.Function):
    """logits = x W^T and the fused softmax cross-entropy, `mc` token rows at a time.

    Each chunk's logits go into ONE reused [mc, Vp] buffer small enough to stay in the 256 MB
    MALL (Infinity Cache), the fused xent turns it into the gradient in place, and only the
    gradient chunk is written to the full [M, Vp] dlogits buffer in HBM that the backward GEMMs
    read. The whole-tensor path writes the logits to HBM and reads them back (13.2 GB of the
    GPT-2 bench step's traffic); here that round trip was meant to stay in the cache.
    Measured at the GPT-2 bench shape (profiles/r2_lmhead_chunk_probe.log): whole GEMM + xent
    6.6 ms; chunked 9.8-11.3 ms for 1k-8k-row chunks — the chunk GEMMs alone lose 12-57 % to the
    one big GEMM and the cache does not absorb the rest. Hence opt-in (config lmhead_chunk)."""

    @staticmethod
    def forward(ctx, x2, w, targets, vocab, nvalid, mc):
        M, Vp = x2.shape[0], w.shape[0]
        C = native()
        d = torch.empty(M, Vp, device=x2.device, dtype=torch.bfloat16)
        rows = torch.empty(M, device=x2.device, dtype=torch.float32)
        buf = _chunk_buf(mc, Vp, x2.device)
        for i in range(0, M, mc):
            n = min(mc, M - i)
            b = buf[:n]
            torch.matmul(x2[i:i + n], w.t(), out=b)
            r = C.xent_fused(b, targets[i:i + n], nvalid, vocab)
            rows[i:i + n].copy_(r)
            d[i:i + n].copy_(b)
        ctx.save_for_backward(x2, w)
        ctx.d = d
        return rows.sum() / nvalid

    @staticmethod
    def backward(ctx, dloss):
        from .linear import _param_grads, mm

        x2, w = ctx.saved_tensors
        d, ctx.d = ctx.d, None
        native().xent_rescale(d, dloss.float().reshape(1).contiguous())
        dx = mm(d, w) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw, _ = _param_grads(d, x2, w, None, True, False)
        return dx, dw, None, None, None, None


def lm_head_cross_entropy(x, w, targets, vocab: int, chunk: int | None = None):
    """Mean cross-entropy of logits = x @ w^T over the first `vocab` columns (w [Vp, K] may be
    padded). On the GPU with `chunk` rows (default: config ``lmhead_chunk``) per GEMM + xent pass;
    chunk 0 (or CPU tensors) = the unchunked ``cross_entropy(linear(x, w))``."""
    from .linear import linear

    x2 = x.reshape(-1, x.shape[-1])
    t = targets.reshape(-1)
    mc = config.get().lmhead_chunk if chunk is None else chunk
    Vp = w.shape[0]
    if (mc and use_native(x2) and torch.is_grad_enabled() and x2.dtype == torch.bfloat16 and Vp % 8 == 0
            and Vp <= 57344 and x2.shape[0] > mc):
        t = t.contiguous().long()
        nvalid = (t >= 0).sum().clamp_min(1).to(torch.float32).reshape(1)
        return _LMHeadXEnt.apply(x2.contiguous(), w, t, vocab, nvalid, mc)
    return cross_entropy(linear(x2, w), t, vocab=vocab)

