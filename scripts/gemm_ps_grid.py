"""gemm_ps tiles-per-workgroup sweep at the GPT-2 shapes: persistent (one workgroup per CU) vs
k tiles per workgroup vs one tile per workgroup (workgroup turnover: a finished workgroup's stores
drain while the next one on that CU computes). Correctness of each grid checked first."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402
from gemm_ps_bench import timeit  # noqa: E402

C = native()
M = 65536
for name, n, k in [("qkv", 2304, 768), ("fc", 3072, 768), ("proj", 768, 768), ("dg_fc2", 3072, 768)]:
    a = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
    c = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
    tiles = (M // 256) * (n // 256)
    grids = [256, 512, 768, tiles // 2, tiles]
    ref = a[:512].float() @ b.float().t()
    for g in grids:
        c.fill_(float("nan"))
        C.gemm_ps(a, b, c, grid_cap=g)
        torch.cuda.synchronize()
        full = (a.float() @ b.float().t()) if g == grids[0] else None
        err = (c[:512].float() - ref).abs().max().item()
        assert err < 2e-2 * ref.abs().max().item() and not torch.isnan(c).any().item(), (name, g, err)
    ts = timeit([lambda g=g: C.gemm_ps(a, b, c, grid_cap=g) for g in grids] + [lambda: F.linear(a, b)])
    fl = 2.0 * M * n * k
    print(f"{name:7s} " + "  ".join(f"grid {g}: {t:6.1f} us" for g, t in zip(grids, ts[:-1])) +
          f"  | library {ts[-1]:6.1f} us", flush=True)
