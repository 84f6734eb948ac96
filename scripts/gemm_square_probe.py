"""Hand-written gemm_nt vs the library at square sizes (where the per-tile prologue/epilogue is
amortised over a long K loop): separates the kernel's main-loop efficiency from the small-K tile
overhead of the GPT-2 shapes. Random operands, median of 10."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
for n in (4096, 8192):
    a = torch.rand(n, n, device="cuda", dtype=torch.bfloat16) * 2 - 1
    b = torch.rand(n, n, device="cuda", dtype=torch.bfloat16) * 2 - 1
    c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
    res = {}
    for name, fn in (("library", lambda: F.linear(a, b)), ("gemm_nt", lambda: C.gemm_nt(a, b, c))):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(10):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        res[name] = ts[5]
    fl = 2.0 * n ** 3
    print(f"{n}^3: library {res['library'] * 1e3:8.1f} us ({fl / res['library'] / 1e9:6.0f} TF)  "
          f"gemm_nt {res['gemm_nt'] * 1e3:8.1f} us ({fl / res['gemm_nt'] / 1e9:6.0f} TF)", flush=True)
