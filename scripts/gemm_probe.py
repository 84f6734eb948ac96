"""Times the GPT-2-small bench GEMMs (forward, dgrad, wgrad; B*T = 65536 tokens) as the
autograd graph issues them, hot (back-to-back) and cold (a 1 GiB write between calls evicts
L2 and the 256 MB Infinity Cache, as in a real step). TunableOp settings come from the env.

    python scripts/gemm_probe.py [tokens]
"""
import os
import sys

import torch
import torch.nn.functional as F

M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = "cuda"
bf = torch.bfloat16
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
SHAPES = [("qkv", 2304, 768, True), ("proj", 768, 768, False), ("fc", 3072, 768, False), ("fc2", 768, 3072, False),
          ("lm", 50304, 768, False)]


def bench(fn, cold, it=10):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(it):
        if cold:
            flush.fill_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


tag = os.environ.get("PROBE_TAG", "")
SPLITS = [int(v) for v in os.environ.get("PROBE_SPLITS", "").split(",") if v]
tot = {False: 0.0, True: 0.0}
for name, N, K, has_bias in SHAPES:
    x = torch.randn(M, K, device=dev, dtype=bf)
    w = torch.randn(N, K, device=dev, dtype=bf) * 0.02
    b = torch.zeros(N, device=dev, dtype=bf) if has_bias else None
    dy = torch.randn(M, N, device=dev, dtype=bf)
    ops = {"fwd": lambda: F.linear(x, w, b), "dgrad": lambda: dy.mm(w), "wgrad": lambda: dy.t().mm(x)}
    for S in SPLITS:  # split-M wgrad: batched partial products, then a sum over the splits
        ops[f"wg/{S}"] = (lambda S=S: torch.bmm(dy.view(S, M // S, N).transpose(1, 2), x.view(S, M // S, K))
                          .sum(0, dtype=torch.float32))
    for op, fn in ops.items():
        fl = 2.0 * M * N * K
        h, c = bench(fn, False), bench(fn, True)
        n = (1 if name == "lm" else 12) * (op in ("fwd", "dgrad", "wgrad"))
        tot[False] += h * n
        tot[True] += c * n
        print(f"{tag:8s} {name:5s} {op:5s} N={N:5d} K={K:4d}  hot {h:8.1f} us ({fl / h / 1e6:6.0f} TF)  "
              f"cold {c:8.1f} us ({fl / c / 1e6:6.0f} TF)", flush=True)
    del x, w, b, dy
print(f"{tag:8s} per-step GEMM total: hot {tot[False] / 1e3:.2f} ms  cold {tot[True] / 1e3:.2f} ms", flush=True)
