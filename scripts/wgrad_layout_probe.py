"""Probe: formulations of the GPT-2 LM-head weight gradient dW[V, C] = dY[M, V]^T X[M, C]
(M = 65536 tokens, V = 50304, C = 768) on the library GEMMs. Prints median ms of each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402
from distributedvolunteercomputing_amd.ops.linear import wgrad  # noqa: E402

dev = torch.device("cuda", 0)
M, V, C = 65536, 50304, 768
dy = (torch.randn(M, V, device=dev) * 0.01).to(torch.bfloat16)
x = torch.randn(M, C, device=dev).to(torch.bfloat16)
g = torch.zeros(V, C, device=dev, dtype=torch.bfloat16)
gT = torch.empty(C, V, device=dev, dtype=torch.bfloat16)


def t(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[2]


variants = {
    "current wgrad() (split-M bmm + reduce)": lambda: wgrad(dy, x, out=g, accumulate=True),
    "one GEMM, addmm_ beta=1": lambda: g.addmm_(dy.t(), x),
    "one GEMM, mm into fresh": lambda: torch.mm(dy.t(), x),
    "transposed: X^T dY -> [C, V]": lambda: torch.mm(x.t(), dy, out=gT),
    "transposed + add^T into grad": lambda: g.add_(torch.mm(x.t(), dy).t()),
    "split-M 2 bmm": lambda: torch.bmm(dy.view(2, M // 2, V).transpose(1, 2), x.view(2, M // 2, C)),
    "split-M 8 bmm": lambda: torch.bmm(dy.view(8, M // 8, V).transpose(1, 2), x.view(8, M // 8, C)),
}
for k, fn in variants.items():
    ms = t(fn)
    print(f"{k:42s} {ms:7.3f} ms  {2 * M * V * C / ms / 1e9:7.1f} TF/s", flush=True)
