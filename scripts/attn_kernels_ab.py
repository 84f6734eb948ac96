"""Runs the attention kernels of every variant several times (for rocprofv3 --kernel-trace:
per-kernel times of each template instance, distinguishable by their template arguments)."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native
C = native()
B, H, T, D = 64, 12, 1024, 64
qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16)
dO = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
o, l = C.attn_fwd(qkv, 0.125)
for rnd in range(3):
    for v in [(3, 1, 0), (3, 1, 1), (2, 0, 0), (2, 1, 1)]:
        C.attn_set_variant(*v)
        for _ in range(3):
            C.attn_fwd(qkv, 0.125)
            C.attn_bwd(qkv, o, dO, l, 0.125)
torch.cuda.synchronize()
