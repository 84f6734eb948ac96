"""Gradient-compression kernels alone, for counter runs: top-k 1% with error feedback and PowerSGD
rank 4 (lazy error feedback) over a flat bf16 gradient of 16 Linear(4096, 4096) layers
(268M parameters, the Llama-3-8B projection shape), 4 rounds each, single peer.

    python scripts/compress_only.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedvolunteercomputing_amd.parallel.compression import PowerSGDCompressor, TopKCompressor  # noqa: E402
from distributedvolunteercomputing_amd.parallel.flat_params import FlatParams  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = torch.nn.Sequential(*[torch.nn.Linear(4096, 4096, bias=False) for _ in range(16)]).to(dev, torch.bfloat16)
flat = FlatParams(m)
g = (torch.randn(flat.numel, device=dev) * 0.01).to(torch.bfloat16)
topk = TopKCompressor(flat.numel, 0.01, dev)
psgd = PowerSGDCompressor(flat, rank=4, device=dev)
for _ in range(4):
    topk.allreduce_mean(g, None)
    psgd.allreduce_mean(g, None)
torch.cuda.synchronize()
print(f"[compress_only] n={flat.numel} topk ratio={1 / topk.ratio:.1f} psgd ratio={psgd.compression_ratio:.1f}")
