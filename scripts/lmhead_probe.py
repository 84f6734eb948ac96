"""Forward-GEMM layout probe at the GPT-2-small bench shape (65536 tokens): x @ W^T with W stored
[N, K] (the nn.Linear layout, library "TN") against x @ Wt with Wt stored [K, N] ("NN"), cold
(L2 + Infinity Cache flushed between calls), with the committed TunableOp table unless
VCX_TUNABLEOP=off. Prints the median time and the kernel each call ran.

    python scripts/lmhead_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

TUNED = enable_tuned_gemms(0)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

M = 65536
dev = "cuda"
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)


def bench(fn, it=10):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(it):
        flush.fill_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def kname(fn):
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as p:
        fn()
        torch.cuda.synchronize()
    names = [e.key for e in p.key_averages() if "fill" not in e.key.lower()]
    return (names[0] if names else "?")[:70]


print(f"tunableop={TUNED}")
for name, N, K in [("lm", 50304, 768), ("qkv", 2304, 768), ("fc", 3072, 768), ("fc2", 768, 3072), ("proj", 768, 768)]:
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    wt = w.t().contiguous()
    fl = 2.0 * M * N * K
    for lay, fn in [("x@W^T", lambda: F.linear(x, w)), ("x@Wt ", lambda: torch.mm(x, wt)),
                    ("(W@x^T)^T", lambda: torch.mm(w, x.t()))]:
        t = bench(fn)
        print(f"{name:5s} {lay:10s} {t:8.1f} us  {fl / t / 1e9:6.1f} TF/s  {kname(fn)}", flush=True)
    del x, w, wt
