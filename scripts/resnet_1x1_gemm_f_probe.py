"""ResNet-50's 1x1 convolutions (BASELINE config 3, B=128) as GEMMs: the library (what ops.linear runs) against
gemm_f (csrc/kernels/gemm_f.hip, automatic split-K) for the forward Y = X W^T and the input gradient dX = dY W
(gemm_f on the transposed weight), at every shape gemm_f takes (N % 128 == 0, K % 64 == 0, K >= 192).
Median of 5 interleaved rounds x 5 launches; relative error against an fp32 product."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
# (name, rows, cin, cout) per 1x1 convolution
CONVS = [("s1 conv1", 56 * 56, 256, 64), ("s1 conv3", 56 * 56, 64, 256), ("s2 conv1a", 56 * 56, 256, 128),
         ("s2 conv1", 28 * 28, 512, 128), ("s2 conv3", 28 * 28, 128, 512), ("s2 down", 28 * 28, 256, 512),
         ("s3 conv1a", 28 * 28, 512, 256), ("s3 conv1", 14 * 14, 1024, 256), ("s3 conv3", 14 * 14, 256, 1024),
         ("s3 down", 14 * 14, 512, 1024), ("s4 conv1a", 14 * 14, 1024, 512), ("s4 conv1", 7 * 7, 2048, 512),
         ("s4 conv3", 7 * 7, 512, 2048), ("s4 down", 7 * 7, 1024, 2048)]
torch.manual_seed(0)
cases = []
for name, hw, cin, cout in CONVS:
    M = B * hw
    x = torch.randn(M, cin, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(cout, cin, device="cuda", dtype=torch.bfloat16) * cin ** -0.5
    dy = torch.randn(M, cout, device="cuda", dtype=torch.bfloat16)
    for d, (a, bt, nn_, kk, lib) in {
            "fwd": (x, w, cout, cin, lambda x=x, w=w: F.linear(x, w)),
            "dgrad": (dy, w.t().contiguous(), cin, cout, lambda dy=dy, w=w: torch.mm(dy, w))}.items():
        cases.append((name, d, M, nn_, kk, "library", lib))
        if C.gemm_f_supported(M, nn_, kk):
            y = torch.empty(M, nn_, device="cuda", dtype=torch.bfloat16)
            C.gemm_f(a, bt, y)
            ref = a.float() @ bt.float().t()
            torch.cuda.synchronize()
            err = ((y.float() - ref).norm() / ref.norm()).item()
            del ref
            sp = C.gemm_f_splits(M, nn_, kk)
            cases.append((name, d, M, nn_, kk, f"gemm_f s{sp} e{err:.0e}", lambda a=a, bt=bt, y=y: C.gemm_f(a, bt, y)))


def tm(fn, it=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


res = {}
for _ in range(5):
    for c in cases:
        res.setdefault(c[:6], []).append(tm(c[6]))
for c in cases:
    name, d, M, N, K, kind = c[:6]
    t = sorted(res[c[:6]])[2]
    print(f"{name:10s} {d:5s} M={M:6d} N={N:4d} K={K:4d} {kind:18s} {t:8.1f} us {2.0 * M * N * K / t / 1e6:6.0f} TF",
          flush=True)
