"""Default-variant attention timing at the GPT-2-small bench shape (B=64, H=12, T=1024, D=64): forward and
backward medians over 7 rounds x 10 calls, with output checksums so two builds can be compared bit for bit
(a build-flag A/B runs this script once per build, alternating, and compares the JSON lines)."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("VCX_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
B, T, H, D = 64, 1024, 12, 64
torch.manual_seed(0)
qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16)
dO = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
scale = D ** -0.5
fl = 4 * B * H * T * T * D / 2


def tm(fn, it=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


o, lse = C.attn_fwd(qkv, scale)
g = C.attn_bwd(qkv, o, dO, lse, scale)
torch.cuda.synchronize()
f, b = [], []
for _ in range(7):
    f.append(tm(lambda: C.attn_fwd(qkv, scale)))
    b.append(tm(lambda: C.attn_bwd(qkv, o, dO, lse, scale)))
fm, bm = sorted(f)[3], sorted(b)[3]
print(json.dumps({"so": C.__file__, "fwd_ms": round(fm, 4), "bwd_ms": round(bm, 4),
                  "fwd_tflops": round(fl / fm / 1e9, 1), "bwd_tflops": round(2.5 * fl / bm / 1e9, 1),
                  "o_sum": float(o.float().sum()), "g_sum": float(g.float().sum()), "lse_sum": float(lse.sum())}),
      flush=True)
