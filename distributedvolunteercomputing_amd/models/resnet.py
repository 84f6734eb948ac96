"""ResNet-50 for synthetic ImageNet-shaped data (BASELINE.json config 3: "ResNet-50 on
synthetic ImageNet shapes, top-k sparsified gradients + error feedback, 8 peers").

Channels-last bf16. The 1x1 convolutions (about 70 % of the FLOPs) are plain GEMMs on the NHWC
view -- [N*H*W, Cin] x [Cout, Cin]^T -- and run through the framework's linear layer (library
GEMMs picked per shape, split-M weight gradients summed straight into the flat gradient buffer);
stride-2 ones subsample the NHWC view first. The 3x3 convolutions run forward and stride-1 input gradient on
the hand-written gemm_f implicit GEMM (every stage) and, at stages 3 / 4, their weight gradients on gemm_wg; the
stride-2 input gradients, the stage-1/2 weight gradients and the 7x7 stem run MIOpen's NHWC kernels. Train-mode BatchNorm runs fused with its ReLU and the residual add (ops/batchnorm.py,
csrc/kernels/batchnorm.hip). BatchNorm statistics are buffers that the trainers average at every
synchronisation.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import config
from ..ops.batchnorm import bn_act, global_avgpool, stem_maxpool
from ..ops.linear import GradJoin, residual_tap


class Conv1x1(nn.Conv2d):
    """1x1 convolution (no bias) computed as a GEMM on the channels-last layout (same parameter as
    nn.Conv2d, so checkpoints and the flat parameter buffer are unchanged)."""

    def __init__(self, cin, cout, stride=1):
        super().__init__(cin, cout, 1, stride=stride, bias=False)

    def gemm_path(self, x) -> bool:
        """This convolution runs as the native GEMM (so a GradJoin on its input is consumed)."""
        from ..ops.linear import native_linear_ok

        return (x.is_cuda and config.get().resnet_conv1x1 == "gemm" and x.is_contiguous(memory_format=torch.channels_last)
                and native_linear_ok(self.weight))

    def forward(self, x, join=None, deposit=False):
        if not (x.is_cuda and config.get().resnet_conv1x1 == "gemm"
                and x.is_contiguous(memory_format=torch.channels_last)):
            assert join is None
            return super().forward(x)
        from ..ops.linear import linear, subsample_tap

        if self.stride[0] != 1:
            assert not deposit
            if join is not None:  # the input gradient lands in the one conv1 deposited (ops/linear.py GradJoin)
                xh, join = subsample_tap(x, join, self.stride[0]), None
            else:
                xh = x.permute(0, 2, 3, 1)[:, ::self.stride[0], ::self.stride[1], :].contiguous()
        else:
            xh = x.permute(0, 2, 3, 1)  # [N, H, W, C] view of the channels-last storage
        N, H, W, C = xh.shape
        # the [Cout, Cin, 1, 1] parameter itself: its gradient lands in the flat .grad directly
        y = linear(xh.reshape(N * H * W, C), self.weight, join=join, deposit=deposit)
        return y.view(N, H, W, self.out_channels).permute(0, 3, 1, 2)


def _fwd_vcx(imgs, H, W, cin, cout, stride) -> bool:
    """gemm_f's implicit-GEMM convolution takes this shape: every ResNet-50 3x3 convolution (64 / 128 channels on its
    256 x 64 / 256 x 128 tiles, 256+ on 256 x 256 with split-K where few tiles; 1.09-1.38x MIOpen forward and
    stride-1 input gradient at every stage, profiles/r6_conv3x3_fwd.txt)."""
    from ..ops._lib import native

    return config.get().conv3x3_fwd == "vcx" and bool(native().gemm_f_conv3x3_supported(imgs, H, W, cin, cout, stride))


class _Conv3x3(torch.autograd.Function):
    """3x3 convolution (pad 1). Forward and stride-1 input gradient on gemm_f's implicit GEMM
    (csrc/kernels/gemm_f.hip CONV: the patch matrix gathered by the LDS-DMA's per-lane offsets; the input gradient
    as the forward convolution of dy with the flipped, transposed weights) where it measured faster than MIOpen,
    MIOpen's otherwise; the weight gradient on gemm_wg (csrc/kernels/gemm_wg.hip, the patch matrix of x gathered
    while staging), written straight into the parameter's flat .grad when it has one (channels-last
    [Cout][ky][kx][Cin] storage)."""

    @staticmethod
    def forward(ctx, x, w, stride, wg=True):
        from ..ops._lib import native

        ctx.save_for_backward(x, w)
        ctx.stride, ctx.wg = stride, wg
        imgs, cin, H, W = x.shape
        cout = w.shape[0]
        if _fwd_vcx(imgs, H, W, cin, cout, stride):
            Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
            y = torch.empty(imgs, Ho, Wo, cout, device=x.device, dtype=x.dtype)
            native().gemm_f_conv3x3(x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1), y, stride)
            return y.permute(0, 3, 1, 2)  # channels-last NCHW view
        return F.conv2d(x, w, None, stride, 1)

    @staticmethod
    def backward(ctx, dy):
        from ..ops._lib import native

        x, w = ctx.saved_tensors
        s = ctx.stride
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = None
        if ctx.needs_input_grad[0]:
            imgs, cin, H, W = x.shape
            if s == 1 and _fwd_vcx(imgs, H, W, w.shape[0], cin, 1):
                # dx = conv(dy, W') with W'[ci][ky][kx][co] = W[co][ci][2 - ky][2 - kx]: the kernel mirrors its taps
                # (flip_taps), so W' is the transposed weight alone: the [Cout, 9 Cin] channels-last weight matrix
                # transposed by one tiled kernel into tap-major [9][Cin][Cout] (no permute copy, no flip pass)
                dxh = torch.empty(imgs, H, W, cin, device=x.device, dtype=x.dtype)
                cout = w.shape[0]
                wt = native().transpose_bf16(w.permute(0, 2, 3, 1).reshape(cout, 9 * cin)).view(9, cin, cout)
                native().gemm_f_conv3x3(dy.permute(0, 2, 3, 1), wt, dxh, 1, flip_taps=True)
                dx = dxh.permute(0, 3, 1, 2)
            else:
                dx = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                         [True, False, False])[0]
        dw = None
        if ctx.needs_input_grad[1] and not ctx.wg:
            dw = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1]
        elif ctx.needs_input_grad[1]:
            cout = w.shape[0]
            g = w.grad
            dyh, xh = dy.permute(0, 2, 3, 1), x.permute(0, 2, 3, 1)  # contiguous NHWC views
            if (g is not None and g.dtype == w.dtype and g.shape == w.shape
                    and g.is_contiguous(memory_format=torch.channels_last)):
                native().gemm_wg_conv3x3(dyh, xh, g.permute(0, 2, 3, 1).view(cout, -1), True, s)
            else:
                d2 = torch.empty(cout, 3, 3, w.shape[1], device=w.device, dtype=w.dtype)
                native().gemm_wg_conv3x3(dyh, xh, d2.view(cout, -1), False, s)
                dw = d2.permute(0, 3, 1, 2)
        return dx, dw, None, None


class Conv3x3(nn.Conv2d):
    """3x3 convolution, pad 1 (the bottleneck's conv2): nn.Conv2d whose forward and stride-1 input gradient run on
    gemm_f (config.conv3x3_fwd; every ResNet-50 stage) and whose weight gradient runs on gemm_wg where the shape
    tiles (config.conv3x3_wgrad; stages 3 and 4 at B=128)."""

    def __init__(self, cin, cout, stride=1):
        super().__init__(cin, cout, 3, stride=stride, padding=1, bias=False)

    def vcx_wgrad(self, x) -> bool:
        from ..ops._lib import native, use_native

        if not (x.is_cuda and config.get().conv3x3_wgrad == "vcx" and torch.is_grad_enabled()
                and self.weight.requires_grad and self.weight.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
                and use_native(x) and x.is_contiguous(memory_format=torch.channels_last)
                and self.weight.is_contiguous(memory_format=torch.channels_last)):
            return False
        N, C, H, W = x.shape
        # 128 output channels (stage 2) tile but run half-empty 256-row tiles: even with MIOpen there
        # (77-79 vs 78-82 us, config 3 unchanged, profiles/r5_conv3x3_probe.txt) -- 256-multiples only
        return self.out_channels % 256 == 0 and bool(
            native().gemm_wg_conv3x3_supported(self.out_channels, C, N, H, W, self.stride[0]))

    def forward(self, x):
        if self.vcx_wgrad(x):
            return _Conv3x3.apply(x, self.weight, self.stride[0])
        if (x.is_cuda and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16
                and x.is_contiguous(memory_format=torch.channels_last)
                and self.weight.is_contiguous(memory_format=torch.channels_last)
                and _fwd_vcx(x.shape[0], x.shape[2], x.shape[3], x.shape[1], self.out_channels, self.stride[0])):
            return _Conv3x3.apply(x, self.weight, self.stride[0], False)  # MIOpen weight gradient
        return super().forward(x)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = Conv1x1(cin, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = Conv3x3(width, width, stride=stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = Conv1x1(width, cout)
        self.bn3 = nn.BatchNorm2d(cout)
        nn.init.zeros_(self.bn3.weight)  # zero-init residual branch (Goyal et al.)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(Conv1x1(cin, cout, stride=stride), nn.BatchNorm2d(cout))

    def forward(self, x):
        # BatchNorm + ReLU (+ the residual add) as fused HIP passes in train mode (ops/batchnorm.py).
        # Identity shortcut: x feeds conv1 and the residual add, so autograd would sum the two
        # gradients of x in an elementwise pass; the shortcut's gradient goes to conv1's input-gradient
        # GEMM instead, which adds it as its C (beta = 1; ops/linear.py GradJoin)
        # Projection shortcut: conv1's input gradient is left in the join and the shortcut convolution
        # (older node, so its backward runs later) adds its own into it -- beta = 1 at stride 1, a
        # strided in-place add at stride 2 -- instead of autograd's full-size zero fill + slice copy + add
        join = (GradJoin() if (config.get().resnet_join and torch.is_grad_enabled() and self.conv1.gemm_path(x)
                               and (self.down is None or (config.get().resnet_proj_join and self.down[0].gemm_path(x))))
                else None)
        if self.down is None:
            idt = x
        else:
            idt = bn_act(self.down[0](x, join=join), self.down[1], relu=False)
        y = bn_act(self.conv1(x, join=join, deposit=self.down is not None and join is not None), self.bn1)
        y = bn_act(self.conv2(y), self.bn2)
        if join is not None and self.down is None:
            idt = residual_tap(x, join)  # created after conv1's node: its backward runs first
        return bn_act(self.conv3(y), self.bn3, residual=idt)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), n_classes: int = 1000, width: int = 64):
        super().__init__()
        self.stem = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn = nn.BatchNorm2d(width)
        blocks = []
        cin = width
        for i, n in enumerate(layers):
            w = width * (2**i)
            for j in range(n):
                blocks.append(Bottleneck(cin, w, stride=2 if (j == 0 and i > 0) else 1))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, n_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x, y=None):
        x = bn_act(self.stem(x), self.bn)
        x = stem_maxpool(x)  # HIP on channels-last bf16 (ops/batchnorm.py)
        x = self.blocks(x)
        x = global_avgpool(x)
        logits = self.fc(x)
        if y is None:
            return logits
        return F.cross_entropy(logits.float(), y)


def enable_conv_find():
    """MIOpen Find per convolution shape (torch.backends.cudnn.benchmark) for the 3x3 / 7x7
    convolutions, when config.conv_find is on. Process-wide, so the training job / bench that builds
    the ResNet calls it once at setup -- never the model's forward (a forward that flips a
    global made every later convolution of the process, other models and tests included, run Find)."""
    if config.get().conv_find:
        torch.backends.cudnn.benchmark = True


def resnet50(n_classes=1000):
    return ResNet((3, 4, 6, 3), n_classes)


def resnet_tiny(n_classes=10):
    return ResNet((1, 1, 1, 1), n_classes, width=8)
