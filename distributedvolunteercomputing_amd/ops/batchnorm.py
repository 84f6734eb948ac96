"""Train-mode BatchNorm fused with the ReLU after it and the residual add before that ReLU, on
channels-last bf16 activations (csrc/kernels/batchnorm.hip): y = relu(bn(x) [+ residual]).

Forward: one statistics pass (read x), a per-channel finalize (running stats updated in place),
one apply pass (read x [+ residual], write y). With a per-layer workspace (_LayerWS, the default for
modules) the finalize runs inside the apply pass and the backward's inside its dx pass: two launches
per layer and direction instead of three. Backward: one reduction pass (read dy, y, x) and
one input-gradient pass (read dy, mask, x; write dx [and d residual]): the ReLU mask is one bit per
element written by the forward's apply pass (1/16 of the bytes of y, which the backward used to read),
so neither the pre-activation nor y is kept for the backward. On CPU, in fp32 or for unsupported channel counts the
torch composition runs instead (the numerics oracle of tests/test_models_gpu.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import config
from ._lib import grad_buffer, native, use_native


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1)  # a contiguous [N, H, W, C] view of channels-last storage


class _LayerWS:
    """A BatchNorm module's own fp32 [4C] workspace [forward sums | backward sums] and which halves are
    known to be zero on the device. The kernels keep them zero in steady state: the forward's apply pass
    zeroes the backward half and the backward's dx pass the forward half (batchnorm.hip, FIN). Calls out
    of that order -- a forward whose backward never ran, two forwards before their backwards, a second
    backward through a retained graph -- find a half not known to be zero and clear it first (one fill).
    The halves' states follow the launch order on one stream, which a hipGraph capture of a whole
    forward + backward step preserves (the same state before and after the captured step)."""

    __slots__ = ("t", "f_clean", "b_clean")

    def __init__(self, C, device):
        self.t = torch.zeros(4 * C, dtype=torch.float32, device=device)
        self.f_clean = True
        self.b_clean = True

    def before_forward(self):
        if not self.f_clean:
            self.t[: self.t.numel() // 2].zero_()
        self.f_clean, self.b_clean = False, True  # the apply pass zeroes the backward half

    def before_backward(self):
        if not self.b_clean:
            self.t[self.t.numel() // 2:].zero_()
        self.b_clean, self.f_clean = False, True  # the dx pass zeroes the forward half


def _layer_ws(bn: torch.nn.Module, x: torch.Tensor) -> _LayerWS:
    ws = getattr(bn, "_vcx_ws", None)
    if ws is None or ws.t.device != x.device or ws.t.numel() != 4 * x.shape[1]:
        ws = _LayerWS(x.shape[1], x.device)
        object.__setattr__(bn, "_vcx_ws", ws)  # not a parameter / buffer: no state_dict entry
    return ws


class _BNAct(torch.autograd.Function):
    """The statistics kernel finalizes in its last block (running stats, num_batches_tracked); with
    preset flat .grad buffers the backward reduction ADDS dgamma / dbeta into them and autograd gets
    None for gamma / beta (no cast or accumulation kernels per layer)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, run_mean, run_var, eps, momentum, relu, nbt, lws=None):
        C = native()
        xh = _nhwc(x)
        rh = _nhwc(residual) if residual is not None else None
        if lws is not None:
            lws.before_forward()
        y, mean, rstd, scale, mask = C.bn_fwd_train(xh, rh, weight, bias, run_mean, run_var, eps, momentum, relu, nbt,
                                                    lws.t if lws is not None else None)
        ctx.lws = lws
        ctx.save_for_backward(xh, mask if relu else None, mean, rstd, scale)
        ctx.relu, ctx.has_res, ctx.pdtype = relu, residual is not None, weight.dtype
        ctx.params = (weight, bias)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        xh, mask, mean, rstd, scale = ctx.saved_tensors
        weight, bias = ctx.params  # (kept: a retained graph may run this backward again)
        dyh = _nhwc(dy)
        if not dyh.is_contiguous():
            dyh = dyh.contiguous()
        gw = grad_buffer(weight) if ctx.needs_input_grad[1] else None
        gb = grad_buffer(bias) if ctx.needs_input_grad[2] else None
        flat = gw is not None and gb is not None
        lws = ctx.lws
        if lws is not None:
            lws.before_backward()
        dx, dres, dgamma, dbeta = native().bn_bwd(dyh, mask, xh, mean, rstd, scale, ctx.relu, ctx.has_res,
                                                  gw if flat else None, gb if flat else None,
                                                  lws.t if lws is not None else None)
        dx = dx.permute(0, 3, 1, 2)
        dres = dres.permute(0, 3, 1, 2) if ctx.has_res else None
        if flat:  # already added into the flat .grad buffers
            return dx, None, None, dres, None, None, None, None, None, None, None
        dg = dgamma.to(ctx.pdtype) if ctx.needs_input_grad[1] else None
        db = dbeta.to(ctx.pdtype) if ctx.needs_input_grad[2] else None
        return dx, dg, db, dres, None, None, None, None, None, None, None


def bn_act_ok(x: torch.Tensor, bn: torch.nn.BatchNorm2d) -> bool:
    return (config.get().resnet_bn == "fused" and use_native(x) and bn.training and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and bn.affine and bn.weight.dtype == torch.bfloat16
            and bn.track_running_stats and bn.momentum is not None and bool(native().bn_supported(x.shape[1])))


def bn_act(x: torch.Tensor, bn: torch.nn.BatchNorm2d, residual: torch.Tensor | None = None,
           relu: bool = True) -> torch.Tensor:
    """relu(bn(x) + residual) with `bn`'s parameters and running statistics (train mode)."""
    if bn_act_ok(x, bn) and (residual is None or (residual.dtype == x.dtype and residual.shape == x.shape
                                                  and residual.is_contiguous(memory_format=torch.channels_last))):
        nbt = bn.num_batches_tracked
        if nbt is None or nbt.device != x.device or nbt.dtype != torch.long or nbt.numel() != 1:
            nbt = None  # (then counted here, as torch would)
            if bn.num_batches_tracked is not None:
                bn.num_batches_tracked.add_(1)
        lws = _layer_ws(bn, x) if config.get().bn_layer_ws else None
        return _BNAct.apply(x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var, bn.eps, bn.momentum,
                            relu, nbt, lws)
    y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class _MaxPool3s2(torch.autograd.Function):
    """3x3 / stride-2 / pad-1 max-pool (the ResNet stem) on channels-last bf16: a uint8 window index per
    output element (torch stores int64 flat indices) and a gather backward without fill + scatter."""

    @staticmethod
    def forward(ctx, x):
        y, idx = native().maxpool3s2_fwd(_nhwc(x))
        ctx.save_for_backward(idx)
        ctx.hw = (x.shape[2], x.shape[3])
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        dyh = _nhwc(dy)
        if not dyh.is_contiguous():
            dyh = dyh.contiguous()
        return native().maxpool3s2_bwd(dyh, idx, ctx.hw[0], ctx.hw[1]).permute(0, 3, 1, 2)


def stem_maxpool(x: torch.Tensor) -> torch.Tensor:
    """F.max_pool2d(x, 3, 2, 1): the HIP kernels (csrc/kernels/batchnorm.hip) for channels-last bf16 GPU
    tensors with C % 8 == 0, torch otherwise."""
    if (use_native(x) and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _MaxPool3s2.apply(x)
    return F.max_pool2d(x, 3, 2, 1)


class _GlobalAvgPool(torch.autograd.Function):
    """Global average pool of channels-last bf16 [N, C, H, W] -> [N, C]; the backward broadcasts g / (H W) straight
    into a channels-last gradient (csrc/kernels/batchnorm.hip bcast_hw_kernel) instead of torch's expand, divide and
    channels-last copy (59 us vs ~5 at ResNet-50's [128, 2048, 7, 7], scripts/cfg3_copy_sources.py)."""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return x.mean(dim=(2, 3))

    @staticmethod
    def backward(ctx, g):
        H, W = ctx.hw
        return native().bcast_hw_nhwc(g.contiguous(), H, W, 1.0 / (H * W)).permute(0, 3, 1, 2)


def global_avgpool(x: torch.Tensor) -> torch.Tensor:
    """torch.flatten(F.adaptive_avg_pool2d(x, 1), 1): the HIP broadcast backward for channels-last bf16 GPU tensors
    with C % 8 == 0, torch otherwise."""
    if (use_native(x) and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _GlobalAvgPool.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
