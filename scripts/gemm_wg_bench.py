"""Weight-gradient GEMMs at the GPT-2-small bench shapes (65536 tokens), accumulating into a bf16
gradient as the step does: the library path (split-M batched GEMM + fp32 split reduction, the default
of ops/linear.py until round 5) against gemm_wg with 8 and with 4 loader waves. Correctness vs fp32
first, then medians of interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)

import importlib  # noqa: E402

import torch  # noqa: E402

from distributedvolunteercomputing_amd import config  # noqa: E402
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

L = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")
C = native()
dev = torch.device("cuda", 0)
M = int(os.environ.get("TOKENS", "65536"))
SHAPES = [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072)]
LOADERS = [8, 4]
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

cases = []
for name, N, K in SHAPES:
    g = torch.Generator(device=dev).manual_seed(N + K)
    dy = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    gw = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    C.gemm_wg(dy, x, gw, False)
    err = ((gw.float() - ref).abs().max() / ref.abs().max()).item()
    print(f"{name}: gemm_wg max rel err vs fp32 {err:.2e}, splits {C.gemm_wg_supported(N, K, M) and 'default'}", flush=True)
    assert err < 8e-3
    fl = 2.0 * M * N * K

    def lib(dy=dy, x=x, gw=gw):
        with config.override(gemm_wgrad="lib"):
            L.wgrad(dy, x, out=gw, accumulate=True)
    cases.append((name, "library", fl, lib))
    for ld in LOADERS:
        cases.append((name, f"wg ld{ld}", fl, lambda dy=dy, x=x, gw=gw, ld=ld: C.gemm_wg(dy, x, gw, True, 0, ld)))

for _, _, _, fn in cases:
    fn()
torch.cuda.synchronize()
res = {(c[0], c[1]): [] for c in cases}
for rnd in range(7):
    for name, arm, fl, fn in cases:
        e0, e1 = ev(), ev()
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        e1.synchronize()
        res[(name, arm)].append(e0.elapsed_time(e1) / 5 * 1e3)
tot = {}
for (name, arm), ts in res.items():
    ts.sort()
    us = ts[len(ts) // 2]
    fl = next(c[2] for c in cases if c[0] == name)
    tot[arm] = tot.get(arm, 0.0) + us
    print(f"wgrad {name:5s} {arm:10s} {us:8.1f} us  {fl / us / 1e6:6.0f} TF/s  (min {ts[0]:.1f})", flush=True)
print("per layer: " + "  ".join(f"{a} {t:.0f} us" for a, t in tot.items()), flush=True)
