"""Linear layer whose backward computes the weight gradient on a hand-written token-split GEMM.

The weight gradient of a token-major linear layer, dW[N, K] = dY[M, N]^T X[M, K], reduces over
all M = B*T tokens (65536 at the GPT-2 bench shape) into a small output: a single library GEMM
has only (N/256)*(K/256) output tiles (9..36 at GPT-2-small sizes) for 256 CUs and runs at
0.33-0.77 PF/s. The default is the hand-written ``gemm_wg`` (csrc/kernels/gemm_wg.hip: the token
axis split over the CUs, operands read transposed out of LDS, fp32 partials summed by a HIP kernel
directly INTO the flat gradient buffer -- ``p.grad`` is a view of it, see parallel/flat_params.py):
1.17-1.23 PF/s at the GPT-2 shapes (profiles/r5_gemm_wg.txt). The library fallback (other shapes,
``VCX_GEMM_WGRAD=lib``) splits the token axis into S chunks of ONE batched GEMM (S x more tiles in
flight; 1.3-2.3x a single GEMM, scripts/gemm_probe.py) and sums the partials the same way.

Hand-written GEMMs on the default path (round 4, profiles/r4_gemm_ps_bench.txt): the persistent
``gemm_ps`` (csrc/kernels/gemm_ps.hip, nt output stores) runs the GPT-2 MLP's fc + bias + GELU and
fc2 input gradient x gelu' + bias grad (``_MlpGelu``; 342 vs 422 us and 458 vs 541 us against the
library GEMM + pass), and the input gradients of the qkv and attention-output projections (dX = dY
W on W^T, 200 vs 207 us and 72 vs 77 us; ``dgrad_ps_ok``). The other forward GEMMs stay on the
library, where gemm_ps measures 0.86-0.97x (its stores slow the next tile's main loop:
profiles/r4_gemm_ps_diag.txt). ``VCX_GEMM=vcx`` switches the forward and input-gradient GEMMs to
the older tiled ``gemm_nt`` (csrc/kernels/gemm.hip), slower at these shapes (profiles/r2_gemm_nt.txt).
Other shapes go through ``mm``: per GEMM shape, the first call outside graph capture can time the
TunableOp-selected library GEMM (hipBLASLt / rocBLAS, utils/tuning.py) against hipBLASLt with this
process's own per-shape algorithm search (csrc/bindings_lt.cpp). The bias gradient is a HIP
column-sum kernel added into the flat gradient buffer.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


from .. import config
from ._lib import grad_buffer, native, use_native

MIN_ROWS_PER_SPLIT = 2048


def set_gemm_backend(name: str):
    """'vcx' (hand-written gemm_nt where the shape tiles) or 'lib' (library GEMMs only);
    the ``gemm`` field of the runtime config (config.py)."""
    config.update(gemm="lib" if name == "lib" else "vcx")


def gemm_nt_ok(M: int, N: int, K: int, t) -> bool:
    return (config.get().gemm == "vcx" and use_native(t) and t.dtype == torch.bfloat16
            and bool(native().gemm_nt_supported(M, N, K)))


def gemm_nt(a, b, bias=None, out=None):
    """a [M, K] @ b[N, K]^T (+ bias[N]) on the hand-written MFMA kernel (caller checked gemm_nt_ok)."""
    a = a if a.stride(-1) == 1 else a.contiguous()
    out = torch.empty(a.shape[0], b.shape[0], device=a.device, dtype=a.dtype) if out is None else out
    native().gemm_nt(a, b, out, None, bias, None, 1 if bias is not None else 0)
    return out


_ZERO_BIAS: dict = {}


def narrow_gemm_ok(M: int, N: int, K: int, t) -> bool:
    """Y[M, N] = X[M, K] W[N, K]^T with a narrow output on the vision GEMM (csrc/kernels/vision.hip
    gemm_bias_act_kernel, 128 x 64/128 tiles) instead of the library: the ResNet-50 1x1 convolutions
    with 64 output channels at 56^2 (M = 401k: 21.6 vs 34.5 us, 41.8 vs 55.7, 44.1 vs 57.6) and 128 at
    the 401k-row shape (71.4 vs 75.0); at 100k rows or 256+ columns the library is faster
    (profiles/r5_resnet_1x1_probe.txt). Opt-in (config.narrow_gemm = "vision"): inside the config-3 step
    it measured even (8309 / 8293 vs 8321 / 8292 img/s), the probe's gain did not carry over."""
    return (config.get().narrow_gemm == "vision" and ((N <= 64 and M >= 131072) or (N <= 128 and M >= 393216))
            and K % 32 == 0 and use_native(t) and t.dtype == torch.bfloat16 and t.is_contiguous())


def narrow_gemm(a, w):
    """a [M, K] @ w[N, K]^T on the vision GEMM (caller checked narrow_gemm_ok)."""
    from . import vision as V

    zb = _ZERO_BIAS.get((w.shape[0], w.device))
    if zb is None:
        zb = _ZERO_BIAS[(w.shape[0], w.device)] = torch.zeros(w.shape[0], device=w.device)
    return V.gemm_bias_act(a, w.contiguous(), zb, False)


def gemm_f_ok(M: int, N: int, K: int, t) -> bool:
    """Y[M, N] = X[M, K] W[N, K]^T on the hand-written forward GEMM (csrc/kernels/gemm_f.hip) -- opt-in
    (config.gemm_fwd == "vcx"): 0.85-0.93x the library at the GPT-2 shapes (profiles/r6_gemm_f.txt)."""
    return (config.get().gemm_fwd == "vcx" and use_native(t) and t.dtype == torch.bfloat16 and t.is_contiguous()
            and bool(native().gemm_f_supported(M, N, K)))


def gemm_f(a, w, bias=None):
    """a [M, K] @ w[N, K]^T (+ bias) on gemm_f (caller checked gemm_f_ok)."""
    out = torch.empty(a.shape[0], w.shape[0], device=a.device, dtype=a.dtype)
    native().gemm_f(a, w.contiguous(), out, bias)
    return out


def transpose_weight(w):
    """W^T as a contiguous bf16 matrix (HIP transpose; weights only — a few MB)."""
    return native().transpose_bf16(w.contiguous())
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
    # config.gemm_select; measured: no in-step gain (A/B 956 vs 957 samples/s)
    if not (config.get().gemm_select and a.is_cuda and a.dtype == torch.bfloat16 and a.is_contiguous() and b.is_contiguous()):
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


def _splits(M: int, N: int, K: int) -> int:
    if N * K >= 16 * 1024 * 1024:  # big outputs (LM head) already fill the GPU
        if M < config.get().wgrad_big_split_min_m:
            return 1
        s = 4
    elif M >= 262144:
        # the ResNet-50 1x1 convolutions at 56^2 (M = 401k, 64..256 x 64..256 outputs): ~6k rows per
        # split; 16 splits left 25k-row GEMMs on 64 x 16 library tiles (66-125 vs 37-82 us,
        # profiles/r5_resnet_wgrad_probe.txt)
        s = 64
    else:
        s = 16
    while s > 1 and (M % s or M // s < MIN_ROWS_PER_SPLIT):
        s //= 2
    return s


def gemm_wg_ok(M: int, N: int, K: int, t) -> bool:
    """The hand-written weight-gradient GEMM (csrc/kernels/gemm_wg.hip) takes dW[N, K] from M tokens: the
    default (config.gemm_wgrad == "vcx") wherever the output is a few dozen 256 x 256 tiles that need the
    token split -- 1.17-1.23 PF/s at the GPT-2 shapes against the library's 0.81-0.98
    (profiles/r5_gemm_wg.txt). An output of one round of tiles (129..256) runs unsplit: Llama-3-8B's q / o
    projections ([4096, 4096] from 4096 tokens) 129.7 vs 146.5 us on the library; its k / v (4 splits) and
    gate / up / down (896 tiles) lost 5-11 % and stay on the library (profiles/r6_llama_wgrad.txt). The GPT-2
    LM heads ([50304, 768 | 1024], K <= 1024) take gemm_wg with 1..4 splits (config.wgrad_wide).
    Memory: the binding allocates the fp32 split partials [splits, N, K] per call from the caching allocator --
    a transient 618 MB for the GPT-2-small LM head at 4 splits (824 MB at GPT-2-medium), a few MB elsewhere;
    under a hipGraph capture it is one fixed pool allocation."""
    cfg = config.get()
    tiles = ((N + 255) // 256) * (K // 256)
    wide = cfg.wgrad_wide and K <= 1024 and M >= 32768 and tiles > 128
    one_round = 128 < tiles <= 256 and M >= 4096
    return (cfg.gemm_wgrad == "vcx" and use_native(t) and t.dtype == torch.bfloat16
            and (tiles <= 128 or one_round or wide) and (N % 256 == 0 or wide or cfg.wgrad_ragged)
            and bool(native().gemm_wg_supported(N, K, M)))


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False):
    """dW = dy2^T @ x2 ([M, N], [M, K] -> [N, K]); written into / added onto `out` if given."""
    M, N = dy2.shape
    K = x2.shape[1]
    if gemm_wg_ok(M, N, K, dy2) and dy2.stride(1) == 1 and x2.stride(1) == 1 and (out is None or out.is_contiguous()):
        # hand-written transposed-read MFMA GEMM, token-split fp32 partials summed into `out`
        if out is None:
            out = torch.empty(N, K, device=dy2.device, dtype=dy2.dtype)
            accumulate = False
        native().gemm_wg(dy2, x2, out, accumulate)
        return out
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
            # straight into the (flat) .grad; autograd adds nothing
            wgrad(dy2, x2, out=gw.view(N, -1), accumulate=True)
        else:
            dw = wgrad(dy2, x2).view(w.shape)
    if want_b:
        if gb is not None and (N % 8) == 0:
            native().colsum_bf16(dy2, gb)  # HIP column sums added into the flat .grad
        elif (N % 8) == 0:
            db = native().colsum_bf16(dy2)
        else:
            db = dy2.sum(0, dtype=torch.float32).to(dy2.dtype)
    return dw, db


def _w2(w):
    """The [N, K] matrix of a weight: w itself, or the [N, K] view of a 1x1 convolution's [N, K, 1, 1]."""
    return w if w.dim() == 2 else w.view(w.shape[0], -1)


class GradJoin:
    """Hands one extra gradient of a linear layer's input to that layer's backward, which adds it in
    its input-gradient GEMM (beta = 1) instead of autograd adding the two gradients in a separate
    elementwise pass. Made for a residual block whose input x feeds both its first 1x1 convolution
    and the identity shortcut: ``residual_tap(x, join)`` on the shortcut passes its gradient here,
    ``linear(x2d, w, join=join)`` adds it (models/resnet.py). Protocol (one backward pass at a
    time, both sides on the autograd thread): the tap's backward runs first in practice (it becomes
    ready at the block's last BatchNorm, the convolution only at the end of the branch); whichever
    side runs second sees the other's state, so the result is right in either order.

    Projection shortcuts run the other way round: the shortcut's nodes are older than conv1's, so
    conv1's backward runs first and DEPOSITS its input gradient (``linear(..., join=j, deposit=True)``
    returns None for x); the shortcut convolution then adds its own into that buffer -- with beta = 1
    at stride 1, or as a strided in-place add at stride 2 (``subsample_tap``) instead of autograd's
    zero-filled full-size slice gradient plus a full-size add."""

    def __init__(self):
        self.pending = None  # the shortcut's gradient as the [M, K] matrix of the layer input
        self.ran = False     # the layer's backward ran without it (the tap then returns its gradient)

    def take(self):
        g, self.pending = self.pending, None
        return g


class _ResidualTap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, join):
        ctx.join = join
        join.pending, join.ran = None, False
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        join, ctx.join = ctx.join, None
        if join.ran or g.dim() != 4:
            return g, None
        gh = g.permute(0, 2, 3, 1)  # the [N, H, W, C] view the 1x1 convolution's GEMM uses
        if not gh.is_contiguous():
            return g, None
        join.pending = gh.reshape(-1, gh.shape[-1])
        return None, None


def residual_tap(x: torch.Tensor, join: GradJoin) -> torch.Tensor:
    """x itself (a view), whose gradient goes to ``join`` (channels-last 4-D x) instead of autograd."""
    return _ResidualTap.apply(x, join)


class _SubsampleTap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, join, s):
        ctx.join, ctx.s = join, s
        ctx.full = (x.shape[0], x.shape[2], x.shape[3], x.shape[1])  # N, H, W, C
        join.ran = False
        xh = x.permute(0, 2, 3, 1)
        ctx.hip = _nhwc_hip_ok(xh)
        if ctx.hip:  # csrc/kernels/batchnorm.hip subsample_kernel: 16-B lanes (torch's strided copy: ~1.4 TB/s)
            return native().subsample_nhwc(xh, s)
        return xh[:, ::s, ::s, :].contiguous()

    @staticmethod
    def backward(ctx, g):
        join, ctx.join = ctx.join, None
        s, (N, H, W, C) = ctx.s, ctx.full
        base = join.take()
        if base is not None and base.is_contiguous() and base.numel() == N * H * W * C:
            full = base.view(N, H, W, C)
            # conv1's deposited input gradient: only the strided quarter moves
            if ctx.hip and g.is_contiguous() and _nhwc_hip_ok(g) and full.dtype == g.dtype:
                native().subsample_add_nhwc(full, g, s)
            else:
                full[:, ::s, ::s, :].add_(g)
        else:
            join.ran = True
            full = g.new_zeros(N, H, W, C)
            full[:, ::s, ::s, :] = g
        return full.permute(0, 3, 1, 2), None, None


def _nhwc_hip_ok(t: torch.Tensor) -> bool:
    """A contiguous NHWC bf16 GPU tensor the strided-shortcut kernels take (C % 8 == 0, 16-B aligned)."""
    return (use_native(t) and t.dtype == torch.bfloat16 and t.dim() == 4 and t.is_contiguous() and t.shape[3] % 8 == 0
            and t.data_ptr() % 16 == 0)


def subsample_tap(x: torch.Tensor, join: GradJoin, stride: int) -> torch.Tensor:
    """The contiguous [N, H/s, W/s, C] subsample of channels-last 4-D x (a stride-s 1x1 convolution's
    input); its backward adds the gradient into the input gradient conv1 deposited in ``join``."""
    return _SubsampleTap.apply(x, join, stride)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, bias_grad_elsewhere=False, join=None, deposit=False):
        # w: [N, K], or a 1x1 convolution's [N, K, 1, 1] weight itself (not a view of it: its gradient
        # then goes straight into the parameter's flat .grad, no view-backward + accumulation pass)
        ctx.save_for_backward(x, w)
        # bias_grad_elsewhere: the sole consumer of y computes the bias gradient itself (column
        # sums it already has at hand) and returns it for the same bias tensor
        ctx.has_bias = b is not None and not bias_grad_elsewhere
        ctx.bias = b
        ctx.join, ctx.deposit = join, deposit
        if deposit:
            join.pending, join.ran = None, False
        x2 = x.reshape(-1, x.shape[-1])
        w = _w2(w)
        if gemm_nt_ok(x2.shape[0], w.shape[0], x2.shape[1], x2):
            return gemm_nt(x2, w, b).view(*x.shape[:-1], w.shape[0])
        if gemm_f_ok(x2.shape[0], w.shape[0], x2.shape[1], x2) and (b is None or b.is_contiguous()):
            return gemm_f(x2, w, b).view(*x.shape[:-1], w.shape[0])
        if b is None and narrow_gemm_ok(x2.shape[0], w.shape[0], x2.shape[1], x2):
            return narrow_gemm(x2, w).view(*x.shape[:-1], w.shape[0])
        return mm(x2, w, trans_b=True, bias=b).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, w_param = ctx.saved_tensors
        w = _w2(w_param)
        N, K = w.shape
        dy2 = dy.reshape(-1, N)
        x2 = x.reshape(-1, K)
        dy2 = dy2.contiguous()
        dx = None
        join, ctx.join = ctx.join, None
        deposit = ctx.deposit
        if deposit:  # conv1 of a projection-shortcut block: runs first, leaves dx for the shortcut
            join, depo = None, join
        base = join.take() if join is not None else None
        if join is not None and base is None:
            join.ran = True
        if ctx.needs_input_grad[0] and base is not None and base.shape == (dy2.shape[0], K) and base.is_contiguous():
            # the shortcut's gradient is the C of this GEMM (beta = 1): no separate add pass
            dx = base.addmm_(dy2, w).view(x.shape)
        elif base is not None:
            dx = (mm(dy2, w) + base).view(x.shape) if ctx.needs_input_grad[0] else None
        elif ctx.needs_input_grad[0]:
            if gemm_nt_ok(dy2.shape[0], K, N, dy2):
                dx = gemm_nt(dy2, transpose_weight(w)).view(x.shape)
            elif gemm_f_ok(dy2.shape[0], K, N, dy2):
                dx = gemm_f(dy2, transpose_weight(w)).view(x.shape)
            elif narrow_gemm_ok(dy2.shape[0], K, N, dy2):
                dx = narrow_gemm(dy2, transpose_weight(w)).view(x.shape)
            elif dgrad_ps_ok(dy2.shape[0], K, N, dy2):
                # dX = dY W on the persistent hand-written GEMM (B = W^T, a few MB): faster than the
                # library at the GPT-2 attention shapes (profiles/r4_gemm_ps_bench.txt: dg_qkv, dg_proj)
                dx = torch.empty(dy2.shape[0], K, device=dy2.device, dtype=dy2.dtype)
                native().gemm_ps(dy2, transpose_weight(w), dx)
                dx = dx.view(x.shape)
            else:
                dx = mm(dy2, w).view(x.shape)
        if deposit and dx is not None and not depo.ran and dx.is_contiguous():
            depo.pending, dx = dx.view(-1, K), None
        want_w = bool(ctx.needs_input_grad[1])
        want_b = bool(ctx.has_bias and ctx.needs_input_grad[2])
        bias, ctx.bias = ctx.bias, None
        w = w_param  # gradients are formed for the parameter's own shape
        flat_w = w.grad is not None and w.grad.is_contiguous() and w.grad.dtype == w.dtype
        flat_b = (not want_b) or grad_buffer(bias) is not None
        # config.async_wgrad: measured slower (951 vs 966-971 samples/s)
        if config.get().async_wgrad and dy2.is_cuda and flat_w and flat_b and (want_w or want_b):
            # only when every result lands in a flat .grad buffer (nothing is returned to autograd)
            main = torch.cuda.current_stream(dy2.device)
            side = _side_stream(dy2.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                _param_grads(dy2, x2, w, bias, want_w, want_b)
            dy2.record_stream(side)  # keep the inputs' memory until the side stream is done with it
            x2.record_stream(side)
            _queue_join(main, side, dy2.device)
            return dx, None, None, None, None, None
        dw, db = _param_grads(dy2, x2, w, bias, want_w, want_b)
        return dx, dw, db, None, None, None


def native_linear_ok(w: torch.Tensor) -> bool:
    """True when linear(x, w, ...) runs the native autograd path (where bias_grad_elsewhere applies)."""
    return use_native(w) and w.dtype == torch.bfloat16 and torch.is_grad_enabled() and w.requires_grad


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None,
           bias_grad_elsewhere: bool = False, join: GradJoin | None = None, deposit: bool = False) -> torch.Tensor:
    """y = x @ w^T (+ b), x [..., K], w [N, K] (or a 1x1 convolution's [N, K, 1, 1]). With
    bias_grad_elsewhere the backward leaves the bias gradient to y's consumer (e.g.
    ``causal_attention(qkv, bias=b)``), which must then be y's only consumer and return
    d(loss)/d(b) = column sums of dy for the same tensor. ``join``: see GradJoin (deposit = this
    layer's backward leaves its input gradient in the join for a later consumer)."""
    if native_linear_ok(w):
        return _Linear.apply(x, w, b, bias_grad_elsewhere, join, deposit)
    assert join is None, "a GradJoin needs the native linear path (its backward consumes the joined gradient)"
    return F.linear(x, _w2(w), b)


# ---------------------------------------------------------------- fused GPT-2 MLP
def dgrad_ps_ok(M: int, N: int, K: int, t) -> bool:
    """Input gradient dX[M, N] = dY[M, K] W[K, N] on gemm_ps: where it measured faster than the
    library (K <= 2304: the qkv and attention-output projections; at K = 3072 it is 3 % slower)."""
    return (config.get().dgrad_ps and K <= 2304 and use_native(t) and t.dtype == torch.bfloat16
            and t.is_contiguous() and bool(native().gemm_ps_supported(M, N, K, 0)))


def gemm_ps_ok(M: int, N: int, K: int, epi: int, t) -> bool:
    """The persistent store-overlapped GEMM (csrc/kernels/gemm_ps.hip) takes this shape/epilogue."""
    return (config.get().mlp == "fused" and use_native(t) and t.dtype == torch.bfloat16
            and bool(native().gemm_ps_supported(M, N, K, epi)))


class _MlpGelu(torch.autograd.Function):
    """y = gelu_tanh(x W1^T + b1) W2^T with the two memory-bound MLP passes folded into GEMM epilogues:
    forward  fc:  one GEMM writes pre = x W1^T + b1 AND act = gelu(pre) (no bias_gelu pass);
    backward fc2-dgrad: one GEMM writes dpre = (dy W2) * gelu'(pre) and reduces db1 = sum dpre
             in its epilogue (no bias_gelu_bwd pass, dact never hits HBM).
    `ps`: those two GEMMs run gemm_ps (persistent, nt stores; 0.81x and 0.85x the time of the library
    GEMM + pass, profiles/r4_gemm_ps_bench.txt) and the other MLP GEMMs the library; otherwise all
    four run the tiled gemm_nt (VCX_GEMM=vcx)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, ps):
        C = native()
        x2 = x.reshape(-1, x.shape[-1])
        M, F_ = x2.shape[0], w1.shape[0]
        pre = torch.empty(M, F_, device=x.device, dtype=x.dtype)
        act = torch.empty_like(pre)
        if ps:
            # `pre` holds gelu'(pre) (epilogue 5): the backward needs pre only for gelu', and the forward
            # already has sigmoid(2u) (VCX_MLP_GRAD_FWD=0: store pre, gelu' in the backward's epilogue 4)
            C.gemm_ps(x2, w1, pre, act, b1, None, 5 if config.get().mlp_grad_fwd else 2)
            y = gemm_f(act, w2) if gemm_f_ok(M, w2.shape[0], F_, act) else mm(act, w2, trans_b=True)
        else:
            C.gemm_nt(x2, w1, pre, act, b1, None, 2)
            y = gemm_nt(act, w2)
        ctx.save_for_backward(x2, w1, b1, w2, pre, act)
        ctx.xshape = x.shape
        ctx.ps = ps
        ctx.grad_fwd = bool(ps and config.get().mlp_grad_fwd)
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x2, w1, b1, w2, pre, act = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        M, F_ = pre.shape
        gb = grad_buffer(b1) if ctx.needs_input_grad[2] else None
        # the bias gradient's fp32 column sums: a zero-at-rest buffer per (size, device, stream) that the add into
        # the flat .grad zeroes again (no fill launch per layer), a fresh zero tensor when the sums are returned
        cs = _colsum_buffer(F_, dy.device) if gb is not None else torch.zeros(F_, device=dy.device, dtype=torch.float32)
        dpre = torch.empty_like(pre)
        if ctx.ps:
            C.gemm_ps(dy2, transpose_weight(w2), dpre, pre, None, cs, 6 if ctx.grad_fwd else 4)
        else:
            C.gemm_nt(dy2, transpose_weight(w2), dpre, pre, None, cs, 3)
        dw2, _ = _param_grads(dy2, act, w2, None, ctx.needs_input_grad[3], False)
        dw1, _ = _param_grads(dpre, x2, w1, None, ctx.needs_input_grad[1], False)
        db1 = None
        if ctx.needs_input_grad[2]:
            if gb is not None:
                C.add_f32_into_bf16(cs, gb, True, True)
            else:
                db1 = cs.to(b1.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (mm(dpre, w1) if ctx.ps else gemm_nt(dpre, transpose_weight(w1))).view(ctx.xshape)
        return dx, dw1, db1, dw2, None


_COLSUM = {}


def _colsum_buffer(n: int, device) -> torch.Tensor:
    """Zero-at-rest fp32 [n] on `device` for the current stream: the GEMM epilogue adds column sums into it and
    add_f32_into_bf16(..., zero_src=True) leaves it zeroed again (uses on one stream are ordered)."""
    key = (n, device, torch.cuda.current_stream(device).cuda_stream)
    buf = _COLSUM.get(key)
    if buf is None:
        buf = _COLSUM[key] = torch.zeros(n, device=device, dtype=torch.float32)
    return buf


def mlp_gelu_ok(x, w1, w2) -> bool:
    return _mlp_mode(x, w1, w2) is not None


def _mlp_mode(x, w1, w2):
    """'ps' (fused epilogues on gemm_ps), 'nt' (everything on gemm_nt) or None (library + passes)."""
    if not (native_linear_ok(w1) and x.dtype == torch.bfloat16):
        return None
    M = x.numel() // x.shape[-1]
    F_, C_ = w1.shape
    if gemm_ps_ok(M, F_, C_, 2, x) and gemm_ps_ok(M, F_, w2.shape[0], 4, x):
        return "ps"
    if (gemm_nt_ok(M, F_, C_, x) and gemm_nt_ok(M, w2.shape[0], F_, x) and gemm_nt_ok(M, C_, w2.shape[0], x)
            and gemm_nt_ok(M, F_, w2.shape[0], x)):
        return "nt"
    return None


def mlp_gelu(x, w1, b1, w2):
    """gelu_tanh(x W1^T + b1) W2^T (GPT-2 MLP without the fc2 bias, which the following fused
    add + LayerNorm applies)."""
    mode = _mlp_mode(x, w1, w2)
    if mode is not None:
        return _MlpGelu.apply(x, w1, b1, w2, mode == "ps")
    from .activations import bias_gelu

    return linear(bias_gelu(linear(x, w1), b1), w2)
