import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native
C = native()
for (B, T, H) in [(8, 1024, 12), (1, 128, 1), (1, 256, 1), (4, 512, 4), (64, 1024, 12)]:
    torch.manual_seed(5)
    qkv = torch.randn(B, T, 3, H, 64, device="cuda").to(torch.bfloat16)
    for v in [(2, 0), (2, 1), (3, 1)]:
        C.attn_set_variant(*v)
        o0, l0 = C.attn_fwd(qkv, 0.125)
        nd_tot = 0
        for rep in range(5):
            o1, l1 = C.attn_fwd(qkv, 0.125)
            d = (o1 != o0)
            nd = int(d.sum())
            nd_tot += nd
            if nd and rep == 0:
                idx = d.nonzero()
                tq = idx[:, 1]
                print(f"  B{B} T{T} H{H} v{v}: {nd} differ; t range {int(tq.min())}-{int(tq.max())}, "
                      f"t%128 hist {torch.bincount((tq % 128) // 32, minlength=4).tolist()}, "
                      f"tile(t//128) hist {torch.bincount(tq // 128).tolist()[:8]}, "
                      f"d hist {torch.bincount(idx[:, 3] // 16, minlength=4).tolist()}, "
                      f"max diff {(o1.float() - o0.float()).abs().max().item():.3e}, lse differ {int((l1 != l0).sum())}",
                      flush=True)
        print(f"B{B} T{T} H{H} v{v}: total differing over 5 reps {nd_tot}", flush=True)
