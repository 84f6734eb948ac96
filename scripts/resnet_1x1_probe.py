"""ResNet-50 1x1 convolutions as NHWC GEMMs (BASELINE config 3, B=128) -- the library path the step takes
(torch mm / F.linear with the shipped TunableOp table) against the hand-written vision GEMM
(csrc/kernels/vision.hip gemm_bias_act_kernel: 128 x 64/128 tiles, no bias) for the forward Y = X W^T and
the input gradient dX = dY W. Prints us per call and TB/s of the operand + output bytes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import vision as V  # noqa: E402

dev = torch.device("cuda", 0)
B = 128
# (H, Cin, Cout): conv1 (in -> width), conv3 (width -> 4 width), downsample (in -> 4 width) per stage
SHAPES = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 512, 128), (28, 128, 512), (56, 256, 128),
          (14, 1024, 256), (14, 256, 1024), (28, 512, 256), (7, 2048, 512), (7, 512, 2048), (14, 1024, 512)]


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


for H, cin, cout in SHAPES:
    M = B * H * H
    x = torch.randn(M, cin, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(cout, cin, device=dev) / cin ** 0.5).to(torch.bfloat16)
    dy = torch.randn(M, cout, device=dev, dtype=torch.bfloat16)
    wt = w.t().contiguous()  # [cin, cout]: dX = dY W as a NT GEMM dY . (W^T)^T
    zb_o, zb_i = torch.zeros(cout, device=dev), torch.zeros(cin, device=dev)
    for what, lib, vcx, nbytes, ref in (
            ("fwd  ", lambda: torch.nn.functional.linear(x, w), lambda: V.gemm_bias_act(x, w, zb_o, False),
             2 * (M * cin + M * cout + cin * cout), lambda: x.float() @ w.float().t()),
            ("dgrad", lambda: torch.mm(dy, w), lambda: V.gemm_bias_act(dy, wt, zb_i, False),
             2 * (M * cin + M * cout + cin * cout), lambda: dy.float() @ w.float())):
        r = ref()
        err = float((vcx().float() - r).norm() / r.norm())
        tl, tv = bench(lib), bench(vcx)
        print(f"{what} M={M:6d} K={cin if what == 'fwd  ' else cout:5d} N={cout if what == 'fwd  ' else cin:5d}: "
              f"library {tl:7.1f} us {nbytes / tl / 1e6:5.2f} TB/s | vision GEMM {tv:7.1f} us {nbytes / tv / 1e6:5.2f} TB/s"
              f" | rel err {err:.1e}", flush=True)
