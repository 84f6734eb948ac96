"""A/B of the attention forward staging: two-buffer LDS-DMA (fwd_dma=1, the round-5 default) vs the
3-slot inline-asm LDS-DMA ring (fwd_dma=2) at 2 and 3 waves per SIMD, GPT-2-small bench shape
(B=64, H=12, T=1024, D=64), one process, interleaved rounds, medians; outputs compared bit for bit
with the default (the ring changes the staging only, not the arithmetic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
H, D = 12, 64
torch.manual_seed(0)
qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16)
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


C.attn_set_variant(3, 1, 1, 1)
o_ref, l_ref = C.attn_fwd(qkv, scale)
torch.cuda.synchronize()
variants = [(3, 1), (3, 2), (2, 2), (2, 1)]
for v in variants:
    C.attn_set_variant(v[0], v[1], 1, 1)
    o, l = C.attn_fwd(qkv, scale)
    torch.cuda.synchronize()
    print(f"fwd {v}: max|o - o_default| = {(o.float() - o_ref.float()).abs().max().item():.3e}  "
          f"max|lse - lse_default| = {(l - l_ref).abs().max().item():.3e}", flush=True)
res = {v: [] for v in variants}
for rnd in range(5):
    for v in variants:
        C.attn_set_variant(v[0], v[1], 1, 1)
        res[v].append(tm(lambda: C.attn_fwd(qkv, scale)))
for v, ts in res.items():
    ms = sorted(ts)[len(ts) // 2]
    print(f"fwd (waves/SIMD, staging) {v}: {ms:.4f} ms  {fl / ms / 1e9:7.1f} TF/s  rounds {['%.4f' % x for x in ts]}",
          flush=True)

# backward: bwd_dma bits (1: dQ LDS-DMA two-buffer, 2: dK/dV LDS-DMA two-buffer, 4: dK/dV ring, 8: dQ ring)
dO = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16)
C.attn_set_variant(3, 1, 1, 1)
g_ref = C.attn_bwd(qkv, o_ref, dO, l_ref, scale)
bvars = [1, 5, 8, 12, 3]
for v in bvars:
    C.attn_set_variant(3, 1, v, 1)
    g = C.attn_bwd(qkv, o_ref, dO, l_ref, scale)
    torch.cuda.synchronize()
    print(f"bwd bits {v}: max|dqkv - default| = {(g.float() - g_ref.float()).abs().max().item():.3e}", flush=True)
bres = {v: [] for v in bvars}
for rnd in range(5):
    for v in bvars:
        C.attn_set_variant(3, 1, v, 1)
        bres[v].append(tm(lambda: C.attn_bwd(qkv, o_ref, dO, l_ref, scale)))
for v, ts in bres.items():
    ms = sorted(ts)[len(ts) // 2]
    print(f"bwd bits {v}: {ms:.4f} ms  {2.5 * fl / ms / 1e9:7.1f} TF/s  rounds {['%.4f' % x for x in ts]}", flush=True)
C.attn_set_variant(3, 1, 1, 1)
