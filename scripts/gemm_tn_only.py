"""gemm_tn alone at the fc2 weight-gradient shape (for counter passes): 3 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
M, N, K = 65536, 768, 3072
dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
out = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    native().gemm_tn(dy, x, out, int(os.environ.get("SPLITS", "7")), True)
torch.cuda.synchronize()
print("ok")
