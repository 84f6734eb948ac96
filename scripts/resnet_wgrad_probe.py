"""ResNet-50 1x1-convolution weight gradients with a 64-wide side at config 3 (B=128, M = 401408 rows at 56^2):
dW[N, K] = dY[M, N]^T X[M, K] as the library's split-M batch (S chunks of M, one batched GEMM, fp32 sum) for
several S, in both operand orders (dW or dW^T = X^T dY, transposed back), against the single GEMM.
Prints us per call; the step uses ops/linear.py _splits (S = 16 for these outputs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402

dev = torch.device("cuda", 0)
M = 128 * 56 * 56


def bench(fn, iters=10):
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


def split_bmm(a, b, S):  # a [M, N], b [M, K] -> a^T b [N, K]
    Mi = a.shape[0] // S
    p = torch.bmm(a.view(S, Mi, -1).transpose(1, 2), b.view(S, Mi, -1))
    return p.float().sum(0) if S > 1 else p[0].float()


for N, K in ((64, 64), (256, 64), (64, 256), (128, 256)):
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    nbytes = 2 * M * (N + K)
    row = []
    for S in (1, 4, 16, 64, 256):
        for tr in (False, True):
            fn = (lambda: split_bmm(x, dy, S).t()) if tr else (lambda: split_bmm(dy, x, S))
            err = float((fn() - ref).norm() / ref.norm())
            t = bench(fn)
            row.append(f"S={S:3d}{'T' if tr else ' '} {t:6.1f}us({nbytes / t / 1e6:4.2f}TB/s,{err:.0e})")
    print(f"dW [{N:3d}, {K:3d}] over {M} rows: " + "  ".join(row), flush=True)
