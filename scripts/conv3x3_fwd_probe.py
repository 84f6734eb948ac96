"""ResNet-50 3x3 convolutions (BASELINE config 3, B=128, channels-last bf16): MIOpen (Find on) against gemm_f's
implicit-GEMM mode (csrc/kernels/gemm_f.hip CONV: the patch matrix of NHWC x gathered by the LDS-DMA's per-lane
source offsets, padding taps read as zeros past the buffer resource) for the forward and, at stride 1, the input
gradient as a forward convolution of dy with the flipped, transposed weights. One line per shape and direction:
us per call, TF/s, relative error of each path against an fp32 convolution."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops._lib import native  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
WAVES = int(os.environ.get("GEMM_F_WAVES", "8"))
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


def rel(a, ref):
    return float((a.float() - ref).norm() / ref.norm())


C = native()
t0 = time.time()
for H, Cin, Cout, s in SHAPES:
    x = torch.randn(B, Cin, H, H, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (3 * Cin ** 0.5)).to(torch.bfloat16).to(memory_format=torch.channels_last)
    Ho = (H - 1) // s + 1
    flops = 2.0 * B * Ho * Ho * Cout * 9 * Cin
    ref = F.conv2d(x.float(), w.float(), stride=s, padding=1).permute(0, 2, 3, 1)
    xh, wh = x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1)
    lib = F.conv2d(x, w, stride=s, padding=1)
    tl = bench(lambda: F.conv2d(x, w, stride=s, padding=1))
    line = f"fwd   {H:3d}^2 {Cin:4d}->{Cout:4d} s{s}: library {tl:7.1f} us {flops / tl / 1e6:6.0f} TF err {rel(lib.permute(0, 2, 3, 1), ref):.1e}"
    if C.gemm_f_conv3x3_supported(B, H, H, Cin, Cout, s):
        y = torch.empty(B, Ho, Ho, Cout, device=dev, dtype=torch.bfloat16)
        C.gemm_f_conv3x3(xh, wh, y, s, None, WAVES)
        tv = bench(lambda: C.gemm_f_conv3x3(xh, wh, y, s, None, WAVES))
        sp = C.gemm_f_splits(B * Ho * Ho, Cout, 9 * Cin)
        line += f" | gemm_f {tv:7.1f} us {flops / tv / 1e6:6.0f} TF err {rel(y, ref):.1e} splits {sp}"
    print(line, flush=True)
    del ref
    if s == 1:
        dy = torch.randn(B, Cout, Ho, Ho, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)

        def lib_dgrad():
            return torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [True, False, False])[0]

        ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [s, s], [1, 1], [1, 1],
                                                  False, [0, 0], 1, [True, False, False])[0].permute(0, 2, 3, 1)
        tl = bench(lib_dgrad)
        line = (f"dgrad {H:3d}^2 {Cin:4d}->{Cout:4d} s{s}: library {tl:7.1f} us {flops / tl / 1e6:6.0f} TF "
                f"err {rel(lib_dgrad().permute(0, 2, 3, 1), ref):.1e}")
        if C.gemm_f_conv3x3_supported(B, Ho, Ho, Cout, Cin, 1):
            # dx = conv(dy, W') with W'[ci][ky][kx][co] = W[co][ci][2 - ky][2 - kx]
            wf = w.flip(2, 3).permute(1, 2, 3, 0).contiguous()
            dyh = dy.permute(0, 2, 3, 1)
            dx = torch.empty(B, H, H, Cin, device=dev, dtype=torch.bfloat16)

            def vcx_dgrad():
                return C.gemm_f_conv3x3(dyh, w.flip(2, 3).permute(1, 2, 3, 0).contiguous(), dx, 1, None, WAVES)

            C.gemm_f_conv3x3(dyh, wf, dx, 1, None, WAVES)
            tv = bench(vcx_dgrad)
            sp = C.gemm_f_splits(B * H * H, Cin, 9 * Cout)
            line += f" | gemm_f+flip {tv:7.1f} us {flops / tv / 1e6:6.0f} TF err {rel(dx, ref):.1e} splits {sp}"
        print(line, flush=True)
        del ref
print(f"done in {time.time() - t0:.0f} s", flush=True)
