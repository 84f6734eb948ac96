"""Runs only the HIP attention fwd+bwd (for rocprofv3 counter collection)."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd import ops
B, H, T, D = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 12, 1024, 64
qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
dO = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    o = ops.causal_attention(qkv); o.backward(dO)
torch.cuda.synchronize()
