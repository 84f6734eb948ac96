"""Default-variant head-major GQA attention timing at the Llama-3-8B shape of config 5 (B=2, Hq=32, Hkv=8,
T=2048, D=128): forward and backward medians over 7 rounds x 10 calls and output checksums, so two builds
can be compared (VCX_AB_ROOT selects the package copy, as scripts/attn_time.py)."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("VCX_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
B, Hq, Hkv, T, D = 2, 32, 8, 2048, 128
torch.manual_seed(0)
q = torch.randn(B, Hq, T, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(B, Hkv, T, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(B, Hkv, T, D, device="cuda", dtype=torch.bfloat16)
dO = torch.randn(B, T, Hq, D, device="cuda", dtype=torch.bfloat16)  # laid out like the output
scale = D ** -0.5
fl = 4 * B * Hq * T * T * D / 2


def tm(fn, it=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


o, lse = C.attn_hm_fwd(q, k, v, scale)
g = C.attn_hm_bwd(q, k, v, o, dO, lse, scale)
torch.cuda.synchronize()
f, b = [], []
for _ in range(7):
    f.append(tm(lambda: C.attn_hm_fwd(q, k, v, scale)))
    b.append(tm(lambda: C.attn_hm_bwd(q, k, v, o, dO, lse, scale)))
fm, bm = sorted(f)[3], sorted(b)[3]
print(json.dumps({"so": C.__file__, "fwd_ms": round(fm, 4), "bwd_ms": round(bm, 4),
                  "fwd_tflops": round(fl / fm / 1e9, 1), "bwd_tflops": round(2.5 * fl / bm / 1e9, 1),
                  "o_sum": float(o.float().sum()), "g_sum": [float(t.float().sum()) for t in g]}), flush=True)
