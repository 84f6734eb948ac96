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

Forward and input-gradient GEMMs go through ``mm``: per GEMM shape, the first call outside graph
capture times the TunableOp-selected library GEMM (hipBLASLt / rocBLAS, utils/tuning.py) against
hipBLASLt with this process's own per-shape algorithm search (csrc/bindings_lt.cpp) and keeps the
faster for the rest of the run (the selections differ by up to ~20% per shape on MI355X). The bias
gradient is a HIP column-sum kernel added into the flat gradient buffer.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

import os

from ._lib import grad_buffer, native, use_native

MIN_ROWS_PER_SPLIT = 2048
_GEMM_SELECT = os.environ.get("VCX_GEMM_SELECT", "0") == "1"  # measured: no in-step gain (A/B 956 vs 957 samples/s)
_CHOICE: dict = {}  # (shapes, layout, bias) -> "torch" | "lt"


def _torch_mm(a, b, trans_a, trans_b, bias):
    if trans_b and not trans_a:  # x @ W^T (+ b): the F.linear / TunableOp GemmAndBias path
        return F.linear(a, b, bias)
    y = torch.mm(a.t() if trans_a else a, b.t() if trans_b else b)
    return y if bias is None else y.add_(bias)


def _lt_mm(a, b, trans_a, trans_b, bias):
    C = native()
    M = a.shape[1] if trans_a else a.shape[0]
    N = b.shape[0] if trans_b else b.shape[1]
    out = torch.empty(M, N, device=a.device, dtype=a.dtype)
    epi = C.LT_EPI_DEFAULT if bias is None else C.LT_EPI_BIAS
    if not C.lt_matmul(a, b, out, trans_a, trans_b, epi, bias):
        return None
    return out


def _time_ms(fn, reps=3):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def mm(a, b, trans_a: bool = False, trans_b: bool = False, bias=None):
    """op(a) @ op(b) (+ bias) for 2-D bf16 GPU tensors, with per-shape library selection."""
    if not (_GEMM_SELECT and a.is_cuda and a.dtype == torch.bfloat16 and a.is_contiguous() and b.is_contiguous()):
        return _torch_mm(a, b, trans_a, trans_b, bias)
    key = (tuple(a.shape), tuple(b.shape), trans_a, trans_b, bias is not None)
    c = _CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return _torch_mm(a, b, trans_a, trans_b, bias)  # no timing inside a capture
        t_torch = _time_ms(lambda: _torch_mm(a, b, trans_a, trans_b, bias))
        c = "torch"
        if _lt_mm(a, b, trans_a, trans_b, bias) is not None:  # runs hipBLASLt's own algorithm search
            if _time_ms(lambda: _lt_mm(a, b, trans_a, trans_b, bias)) < 0.97 * t_torch:
                c = "lt"
        _CHOICE[key] = c
    if c == "lt":
        y = _lt_mm(a, b, trans_a, trans_b, bias)
        if y is not None:
            return y
    return _torch_mm(a, b, trans_a, trans_b, bias)


def gemm_choices() -> dict:
    """{(a.shape, b.shape, trans_a, trans_b, bias): "torch" | "lt"} selected so far."""
    return dict(_CHOICE)


# Big outputs (N*K >= 16M elements) with fewer tokens than this take ONE GEMM that accumulates
# straight into the bf16 .grad (beta = 1) instead of a split-M batch + fp32 partial reduction
_BIG_SPLIT_MIN_M = int(os.environ.get("VCX_WGRAD_BIG_SPLIT_MIN_M", "16384"))


def _splits(M: int, N: int, K: int) -> int:
    if N * K >= 16 * 1024 * 1024:  # big outputs (LM head) already fill the GPU
        if M < _BIG_SPLIT_MIN_M:
            return 1
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
        if out is None:
            return dy2.t().mm(x2)
        if accumulate:
            out.addmm_(dy2.t(), x2)  # one GEMM with beta = 1: no separate product tensor + add pass
        else:
            torch.mm(dy2.t(), x2, out=out)
        return out
    part = torch.bmm(dy2.view(S, M // S, N).transpose(1, 2), x2.view(S, M // S, K))  # [S, N, K]
    if out is None:
        out = torch.empty(N, K, device=dy2.device, dtype=dy2.dtype)
        accumulate = False
    native().splitk_reduce(part, out, accumulate)
    return out


# ---------------------------------------------------------------- side-stream weight gradients
# The weight (and bias) gradient of a layer feeds nothing downstream in the backward pass — only
# the optimizer after it. With VCX_ASYNC_WGRAD=1 (opt-in) those GEMMs + reductions are enqueued
# on a side HIP stream (event fork from the main stream) and joined back once, at the end of the
# backward pass (autograd engine callback), so the compute-bound split-M wgrad GEMMs run beside
# the memory-bound kernels of the next layers' input-gradient chain (LayerNorm / GELU / attention
# backward) instead of after them. Works under hipGraph capture (fork/join become graph edges).
_ASYNC_WGRAD = os.environ.get("VCX_ASYNC_WGRAD", "0") == "1"  # measured slower: 951 vs 966-971 samples/s
_SIDE: dict = {}
_JOIN_PENDING: dict = {}


def _side_stream(dev):
    st = _SIDE.get(dev)
    if st is None:
        st = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return st


def _queue_join(main, side, key):
    """Make `main` wait for `side` when the running backward pass finishes (once per pass)."""
    if _JOIN_PENDING.get(key):
        return
    _JOIN_PENDING[key] = True

    def _join():
        main.wait_stream(side)
        _JOIN_PENDING[key] = False

    torch.autograd.Variable._execution_engine.queue_callback(_join)


def _param_grads(dy2, x2, w, bias, want_w, want_b):
    """(dw, db) to hand autograd: None where the gradient went into a preset flat .grad buffer."""
    dw = db = None
    N = w.shape[0]
    g = w.grad if want_w else None
    gw = g if g is not None and g.is_contiguous() and g.dtype == w.dtype and g.shape == w.shape else None
    gb = grad_buffer(bias) if want_b else None
    if want_w:
        if gw is not None:
            wgrad(dy2, x2, out=gw, accumulate=True)  # straight into the (flat) .grad; autograd adds nothing
        else:
            dw = wgrad(dy2, x2)
    if want_b:
        if gb is not None and (N % 8) == 0:
            native().colsum_bf16(dy2, gb)  # HIP column sums added into the flat .grad
        elif (N % 8) == 0:
            db = native().colsum_bf16(dy2)
        else:
            db = dy2.sum(0, dtype=torch.float32).to(dy2.dtype)
    return dw, db


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, bias_grad_elsewhere=False):
        ctx.save_for_backward(x, w)
        # bias_grad_elsewhere: the sole consumer of y computes the bias gradient itself (column
        # sums it already has at hand) and returns it for the same bias tensor
        ctx.has_bias = b is not None and not bias_grad_elsewhere
        ctx.bias = b
        x2 = x.reshape(-1, x.shape[-1])
        return mm(x2, w, trans_b=True, bias=b).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        N, K = w.shape
        dy2 = dy.reshape(-1, N)
        x2 = x.reshape(-1, K)
        dy2 = dy2.contiguous()
        dx = mm(dy2, w).view(x.shape) if ctx.needs_input_grad[0] else None
        want_w = bool(ctx.needs_input_grad[1])
        want_b = bool(ctx.has_bias and ctx.needs_input_grad[2])
        bias, ctx.bias = ctx.bias, None
        flat_w = w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == w.dtype
        flat_b = (not want_b) or grad_buffer(bias) is not None
        if _ASYNC_WGRAD and dy2.is_cuda and flat_w and flat_b and (want_w or want_b):
            # only when every result lands in a flat .grad buffer (nothing is returned to autograd)
            main = torch.cuda.current_stream(dy2.device)
            side = _side_stream(dy2.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                _param_grads(dy2, x2, w, bias, want_w, want_b)
            dy2.record_stream(side)  # keep the inputs' memory until the side stream is done with it
            x2.record_stream(side)
            _queue_join(main, side, dy2.device)
            return dx, None, None, None
        dw, db = _param_grads(dy2, x2, w, bias, want_w, want_b)
        return dx, dw, db, None


def native_linear_ok(w: torch.Tensor) -> bool:
    """True when linear(x, w, ...) runs the native autograd path (where bias_grad_elsewhere applies)."""
    return use_native(w) and w.dtype == torch.bfloat16 and torch.is_grad_enabled() and w.requires_grad


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None,
           bias_grad_elsewhere: bool = False) -> torch.Tensor:
    """y = x @ w^T (+ b), x [..., K], w [N, K]. With bias_grad_elsewhere the backward leaves the
    bias gradient to y's consumer (e.g. ``causal_attention(qkv, bias=b)``), which must then be
    y's only consumer and return d(loss)/d(b) = column sums of dy for the same tensor."""
    if native_linear_ok(w):
        return _Linear.apply(x, w, b, bias_grad_elsewhere)
    return F.linear(x, w, b)
