"""Runs only the hand-written gemm_nt (and the library GEMM) at two GPT-2 shapes, a few times:
the program profiled by rocprofv3 --pmc for the GEMM counter tables."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
M = 65536
for n, k in ((768, 3072), (3072, 768)):
    a = torch.randn(M, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02
    c = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        C.gemm_nt(a, b, c)
        F.linear(a, b)
torch.cuda.synchronize()
