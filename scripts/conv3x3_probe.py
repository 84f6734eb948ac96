"""ResNet-50 3x3 convolutions (BASELINE config 3, B=128, channels-last bf16): the library (MIOpen, Find on)
against the hand-written implicit-GEMM convolution of csrc/kernels/vision.hip (gemm_bias_act_kernel,
AM_IMPLICIT: the A tile gathered from NHWC x while staging, K-split when few tiles) for the forward and, at
stride 1, the input gradient as a forward convolution of dy with the flipped, transposed weights.
Prints one line per shape and direction: us per call and TF/s of each path, max relative error."""
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from distributedvolunteercomputing_amd.ops._lib import native  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
SHAPES = [(56, 64, 64, 1), (28, 128, 128, 1), (14, 256, 256, 1), (7, 512, 512, 1),
          (56, 128, 128, 2), (28, 256, 256, 2), (14, 512, 512, 2)]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e3)
    return best


C = native()
t0 = time.time()
for H, Cin, Cout, s in SHAPES:
    x = torch.randn(B, Cin, H, H, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)).to(torch.bfloat16).to(memory_format=torch.channels_last)
    Ho = (H + 2 - 3) // s + 1
    flops = 2.0 * B * Ho * Ho * Cout * 9 * Cin
    zb = torch.zeros(Cout, device=dev)
    wt = w.permute(0, 2, 3, 1).reshape(Cout, 9 * Cin).contiguous()
    xh = x.permute(0, 2, 3, 1)
    ref = F.conv2d(x, w, stride=s, padding=1)
    got = C.conv_implicit(xh, wt, zb, Cin, 3, 3, s, 1, False)
    err = float((got.float() - ref.permute(0, 2, 3, 1).float()).norm() / ref.float().norm())
    tl = bench(lambda: F.conv2d(x, w, stride=s, padding=1))
    tv = bench(lambda: C.conv_implicit(xh, wt, zb, Cin, 3, 3, s, 1, False))
    print(f"fwd   {H:3d}^2 {Cin:4d}->{Cout:4d} s{s}: library {tl:7.1f} us {flops / tl / 1e6:6.0f} TF | "
          f"vcx implicit {tv:7.1f} us {flops / tv / 1e6:6.0f} TF | rel err {err:.2e}", flush=True)
    if s == 1:
        dy = torch.randn(B, Cout, Ho, Ho, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        # dx = conv(dy, W') with W'[ci, ky, kx, co] = W[co, ci, 2 - ky, 2 - kx]
        wf = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, 9 * Cout).contiguous()
        dyh = dy.permute(0, 2, 3, 1)
        zb2 = torch.zeros(Cin, device=dev)

        def lib_dgrad():
            return torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [True, False, False])[0]

        ref = lib_dgrad()
        got = C.conv_implicit(dyh, wf, zb2, Cout, 3, 3, 1, 1, False)
        err = float((got.float() - ref.permute(0, 2, 3, 1).float()).norm() / ref.float().norm())
        tl = bench(lib_dgrad)
        tv = bench(lambda: C.conv_implicit(dyh, wf, zb2, Cout, 3, 3, 1, 1, False))
        print(f"dgrad {H:3d}^2 {Cin:4d}->{Cout:4d} s{s}: library {tl:7.1f} us {flops / tl / 1e6:6.0f} TF | "
              f"vcx implicit {tv:7.1f} us {flops / tv / 1e6:6.0f} TF | rel err {err:.2e}", flush=True)

        def lib_wgrad():
            return torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [False, True, False])[1]

        tl = bench(lib_wgrad)
        print(f"wgrad {H:3d}^2 {Cin:4d}->{Cout:4d} s{s}: library {tl:7.1f} us {flops / tl / 1e6:6.0f} TF", flush=True)
# weight gradients: MIOpen vs gemm_wg with the implicit patch operand (csrc/kernels/gemm_wg.hip IMPL) where it tiles
for H, Cin, Cout, s in SHAPES:
    if not C.gemm_wg_conv3x3_supported(Cout, Cin, B, H, H, s):
        continue
    x = torch.randn(B, Cin, H, H, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)).to(torch.bfloat16).to(memory_format=torch.channels_last)
    Ho = (H - 1) // s + 1
    flops = 2.0 * B * Ho * Ho * Cout * 9 * Cin
    dy = torch.randn(B, Cout, Ho, Ho, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)

    def lib_wgrad():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                   [False, True, False])[1]

    out = torch.empty(Cout, 9 * Cin, device=dev, dtype=torch.bfloat16)
    dyh, xh = dy.permute(0, 2, 3, 1), x.permute(0, 2, 3, 1)
    ref = lib_wgrad().float().permute(0, 2, 3, 1).reshape(Cout, -1)
    C.gemm_wg_conv3x3(dyh, xh, out, False, s)
    err = float((out.float() - ref).norm() / ref.norm())
    tl = bench(lib_wgrad)
    tv = bench(lambda: C.gemm_wg_conv3x3(dyh, xh, out, False, s))
    print(f"wgrad {H:3d}^2 {Cin:4d}->{Cout:4d} s{s}: library {tl:7.1f} us {flops / tl / 1e6:6.0f} TF | "
          f"vcx gemm_wg {tv:7.1f} us {flops / tv / 1e6:6.0f} TF | rel err vs library {err:.2e}", flush=True)
print(f"done in {time.time() - t0:.0f} s", flush=True)
