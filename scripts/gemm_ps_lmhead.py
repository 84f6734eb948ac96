"""LM-head input gradient dX = dlogits W at the GPT-2 bench shape (M = 65536, Vp = 50304, C = 768):
the library NN GEMM vs gemm_ps on W^T (a 77 MB transpose per step, timed separately)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402
from gemm_ps_bench import timeit  # noqa: E402

C = native()
M, V, E = 65536, 50304, 768
d = torch.randn(M, V, device="cuda", dtype=torch.bfloat16) * 0.01
w = torch.randn(V, E, device="cuda", dtype=torch.bfloat16) * 0.02
wt = w.t().contiguous()
out = torch.empty(M, E, device="cuda", dtype=torch.bfloat16)
C.gemm_ps(d[:4096], wt, out[:4096])
torch.cuda.synchronize()
ref = d[:4096].float() @ w.float()
err = (out[:4096].float() - ref).abs().max().item()
assert err < 2e-2 * ref.abs().max().item(), err
t = timeit([lambda: torch.mm(d, w), lambda: C.gemm_ps(d, wt, out), lambda: C.transpose_bf16(w)], rounds=3, it=3)
fl = 2.0 * M * V * E
print(f"dg_lm  library {t[0]:8.1f} us ({fl / t[0] / 1e6:5.0f} TF)  gemm_ps {t[1]:8.1f} us ({fl / t[1] / 1e6:5.0f} TF)"
      f"  W^T transpose {t[2]:6.1f} us", flush=True)
