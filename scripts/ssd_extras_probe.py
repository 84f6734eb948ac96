"""MobileNet-SSD's extra 3x3 stride-2 convolutions (conv14_2 .. conv17_2, + bias + ReLU) on one 100-frame chunk:
the vision implicit GEMM the detector runs (conv_implicit, in-kernel split-K) against gemm_f's implicit GEMM (bias only: it had a ReLU flag for this probe) at
every valid K split; relative error against an fp32 convolution. Medians of 5 rounds x 20 calls."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
N = 100
LAYERS = [("conv14_2", 10, 256, 512), ("conv15_2", 5, 128, 256), ("conv16_2", 3, 128, 256), ("conv17_2", 2, 64, 128)]


def tm(fn, it=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


torch.manual_seed(0)
for name, hw, cin, cout in LAYERS:
    x = torch.randn(N, hw, hw, cin, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(cout, 3, 3, cin, device="cuda") / (3 * cin ** 0.5)).to(torch.bfloat16)
    b = torch.randn(cout, device="cuda") * 0.1
    ho = (hw - 1) // 2 + 1
    ref = F.relu(F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), b, 2, 1)).permute(0, 2, 3, 1)
    wt = w.reshape(cout, 9 * cin).contiguous()
    arms = [("vision", lambda: C.conv_implicit(x, wt, b, cin, 3, 3, 2, 1, True))]
    M, K = N * ho * ho, 9 * cin
    y = torch.empty(N, ho, ho, cout, device="cuda", dtype=torch.bfloat16)
    for s in range(1, 17):
        if C.gemm_f_conv3x3_supported(N, hw, hw, cin, cout, 2) and (K // 32) % s == 0 and (K // 32 // s) % 2 == 0 \
                and K // 32 // s >= 6:
            arms.append((f"gemm_f s{s}", lambda s=s: C.gemm_f_conv3x3(x, w, y, 2, b.to(torch.bfloat16), 8, s)))
    res = {a: [] for a, _ in arms}
    errs = {}
    for a, fn in arms:
        out = fn()
        out = y if out is None else out
        torch.cuda.synchronize()
        errs[a] = float((out.float() - ref).norm() / ref.norm())
    for _ in range(5):
        for a, fn in arms:
            res[a].append(tm(fn))
    auto = C.gemm_f_splits(M, cout, K)
    print(f"{name} ({hw}^2 {cin}->{cout}, M={M}, auto split {auto}): " + "  ".join(
        f"{a} {sorted(v)[2]:.1f} us (err {errs[a]:.1e})" for a, v in res.items()), flush=True)
