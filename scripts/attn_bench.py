"""Micro-benchmark of causal attention fwd+bwd at the GPT-2-small bench shape."""
import sys, time, torch, torch.nn.functional as F
B, H, T, D = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 12, 1024, 64
dev = "cuda"
q, k, v = (torch.randn(B, H, T, D, device=dev, dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
do = torch.randn(B, H, T, D, device=dev, dtype=torch.bfloat16)
def run(tag, fn):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(); o = F.scaled_dot_product_attention(q, k, v, is_causal=True) if fn is None else fn_fwd(); e1.record()
        o.backward(do); e2.record(); torch.cuda.synchronize()
        ts.append((e0.elapsed_time(e1), e1.elapsed_time(e2)))
    f = sorted(t[0] for t in ts)[5]; b = sorted(t[1] for t in ts)[5]
    fl = 4 * B * H * T * T * D / 2
    print(f"{tag:24s} fwd {f:7.3f} ms ({fl/f/1e9:6.1f} TF)  bwd {b:7.3f} ms ({2.5*fl/b/1e9:6.1f} TF)", flush=True)
def fn_fwd():
    return F.scaled_dot_product_attention(q, k, v, is_causal=True)
from torch.nn.attention import sdpa_kernel, SDPBackend
for lib in ["aotriton", "ck"]:
    try:
        torch.backends.cuda.preferred_rocm_fa_library(lib)
    except Exception as e:
        print(lib, "unavailable", e); continue
    for be in [SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION]:
        try:
            with sdpa_kernel(be):
                run(f"{lib}/{be.name}", fn_fwd)
        except Exception as e:
            print(lib, be.name, "failed:", str(e)[:200])

# --- hand-written HIP flash attention on the packed layout
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from distributedvolunteercomputing_amd import ops
qkv = torch.randn(B, T, 3, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
dO = torch.randn(B, T, H, D, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    o = ops.causal_attention(qkv); o.backward(dO)
torch.cuda.synchronize()
ts = []
for _ in range(10):
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(); o = ops.causal_attention(qkv); e1.record(); o.backward(dO); e2.record(); torch.cuda.synchronize()
    ts.append((e0.elapsed_time(e1), e1.elapsed_time(e2)))
f = sorted(t[0] for t in ts)[5]; b = sorted(t[1] for t in ts)[5]
fl = 4 * B * H * T * T * D / 2
print(f"{'vcx HIP packed':24s} fwd {f:7.3f} ms ({fl/f/1e9:6.1f} TF)  bwd {b:7.3f} ms ({2.5*fl/b/1e9:6.1f} TF)", flush=True)
