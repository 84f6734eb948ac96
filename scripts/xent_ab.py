"""Fused softmax cross-entropy kernel variants (VCX_XENT_TPB) at the GPT-2-small bench shape
(65536 x 50304 padded logits): time per call and algorithmic bandwidth (one read + one write of
the logits). Each variant runs in its own process (the TPB choice is read once).

    VCX_XENT_TPB=768 python scripts/xent_ab.py
    VCX_XENT_KEEP_E=1 python scripts/xent_ab.py     (one exp per element, norm_act.hip KEEP_E)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
R, V, Vp = 65536, 50257, 50304
logits = torch.randn(R, Vp, device="cuda", dtype=torch.bfloat16)
tgt = torch.randint(0, V, (R,), device="cuda")
nvalid = torch.tensor([float(R)], device="cuda")
ref = logits[:64].float().clone()
C.xent_fused(logits, tgt, nvalid, V)
torch.cuda.synchronize()
p = torch.softmax(ref[:, :V], 1)
p[torch.arange(64), tgt[:64]] -= 1
err = (logits[:64, :V].float() * R - p).abs().max().item()
assert err < 2e-2, err
ts = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        C.xent_fused(logits, tgt, nvalid, V)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) / 5)
t = sorted(ts)[2]
gb = 2 * R * Vp * 2 / 1e9
print(f"VCX_XENT_TPB={os.environ.get('VCX_XENT_TPB', '768')} KEEP_E={os.environ.get('VCX_XENT_KEEP_E', '0')}: {t * 1e3:.1f} us/call, {gb / t:.2f} TB/s algorithmic "
      f"(max err {err:.2e})", flush=True)
