"""Head-major GQA attention at the Llama-3-8B config-5 shape (B=2, Hq=32, Hkv=8, T=2048, D=128):
HIP kernels (attention_hm.hip) vs torch SDPA (AOTriton) fwd and fwd+bwd, median of 10."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedvolunteercomputing_amd import ops  # noqa: E402

B, Hq, Hkv, T, D = 2, 32, 8, 2048, 128
dev = "cuda"
torch.manual_seed(0)
q = torch.randn(B, Hq, T, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(B, Hkv, T, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
do = torch.randn(B, T, Hq, D, device=dev, dtype=torch.bfloat16)
fl = 4 * B * Hq * T * T * D / 2


def tm(fn, it=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def sdpa():
    return F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True).transpose(1, 2)


C = ops.native()
for name, fn, var in (("hip/split", lambda: ops.gqa_attention(q, k, v), 1),
                      ("hip/fused", lambda: ops.gqa_attention(q, k, v), 0), ("sdpa", sdpa, None)):
    if var is not None:
        C.attn_hm_set_variant(var)
    f = tm(lambda: fn())
    fb = tm(lambda: torch.autograd.grad(fn(), (q, k, v), do))
    print(f"{name:9s} fwd {f:7.3f} ms ({fl / f / 1e9:6.1f} TF)  fwd+bwd {fb:7.3f} ms ({3.5 * fl / fb / 1e9:6.1f} TF)",
          flush=True)
