"""The library GEMM and gemm_nt (8 waves) at 4096^3 and the GPT-2
fc shape, a few calls each: the program profiled by scripts/pmc_gemm_cmp.sh."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
for m, n, k in ((4096, 4096, 4096), (65536, 3072, 768)):
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
    c = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        F.linear(a, b)
        C.gemm_nt(a, b, c)
torch.cuda.synchronize()
