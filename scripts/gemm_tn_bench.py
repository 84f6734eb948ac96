"""Weight-gradient GEMMs at the GPT-2-small bench shapes (65536 tokens): the library path
(split-M batched GEMM + split reduction, ops/linear.py) vs the hand-written gemm_tn, both
accumulating into a bf16 gradient. Median of 20 calls; correctness vs fp32 is checked first."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd import config  # noqa: E402
import importlib  # noqa: E402

linear = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")

dev = torch.device("cuda", 0)
M = int(os.environ.get("TOKENS", "65536"))
SHAPES = [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072)]


def med(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


tot = {"lib": 0.0, "vcx": 0.0}
for name, N, K in SHAPES:
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    res = {}
    for be in ("lib", "vcx"):
        with config.override(gemm_wgrad=be):
            out.zero_()
            linear.wgrad(dy, x, out=out, accumulate=True)
            res[be] = out.float().clone()
            us = med(lambda: linear.wgrad(dy, x, out=out, accumulate=True))
        tot[be] += us
        flops = 2.0 * M * N * K
        print(f"{name:5s} N={N:5d} K={K:5d} {be}: {us:8.1f} us  {flops / us / 1e6:7.0f} TF/s"
              + (f"  splits={linear.tn_splits(M, N, K)}" if be == "vcx" else ""), flush=True)
    ref = dy.float().t() @ x.float()
    e = {be: ((r - ref).abs().max() / ref.abs().max()).item() for be, r in res.items()}
    print(f"      max rel err vs fp32: lib {e['lib']:.2e} vcx {e['vcx']:.2e}", flush=True)
print(f"total per layer: lib {tot['lib']:.0f} us, vcx {tot['vcx']:.0f} us")
