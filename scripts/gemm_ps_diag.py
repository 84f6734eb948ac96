"""Where does gemm_ps lose its time once it stores its output? (VERDICT r3 missing #1)

1. Store cache policy A/B at the GPT-2 shapes (M = 65536): plain / nt / sc1 / sc0 sc1 stores against
   the no-store build and the library GEMM (median of interleaved rounds in one process).
2. Per-tile in-kernel s_memtime stamps (thread 0 of every workgroup, cycles): main loop, the wait at
   step 3 of the next tile (the first counted wait that also covers the previous tile's stores),
   and the time to issue the epilogue's stores.

    python scripts/gemm_ps_diag.py
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402
from scripts.gemm_ps_bench import timeit  # noqa: E402

C = native()
dev, bf = "cuda", torch.bfloat16
M = 65536


def stamps_summary(a, b, c, epi, policy, stagger=0):
    grid = 256
    st = torch.zeros(grid, 64, 5, dtype=torch.long, device=dev)
    for _ in range(3):
        C.gemm_ps_diag(a, b, c, epi, policy, None, 0, stagger)
    C.gemm_ps_diag(a, b, c, epi, policy, st, 0, stagger)
    torch.cuda.synchronize()
    s = st.cpu().double()
    tiles = int((s[0, :, 0] > 0).sum())
    s = s[:, :tiles]
    main = (s[:, :, 3] - s[:, :, 0])
    wait3 = (s[:, :, 2] - s[:, :, 1])
    issue = (s[:, :, 4] - s[:, :, 3])
    per_tile = s[:, 1:, 0] - s[:, :-1, 0]
    span = (s[:, -1, 4] - s[:, 0, 0])
    med = lambda t: float(t.flatten().median())  # noqa: E731
    return (f"tiles/wg {tiles}  tile {med(per_tile):8.0f} cyc  main loop {med(main):8.0f}  step-3 wait "
            f"{med(wait3):6.0f} (tile 0: {float(wait3[:, 0].median()):6.0f}, later: {med(wait3[:, 1:]):6.0f})  "
            f"store issue {med(issue):6.0f}  wg span {med(span):9.0f}")


def main():
    shapes = [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("dg_fc2", 3072, 768)]
    for name, n, k in shapes:
        torch.manual_seed(0)
        a = torch.randn(M, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        c = torch.empty(M, n, device=dev, dtype=bf)
        ref = F.linear(a[:4096], b).float()
        for pol in range(4):
            c.zero_()
            C.gemm_ps_diag(a, b, c, 0, pol, None)
            torch.cuda.synchronize()
            err = (c[:4096].float() - ref).abs().max().item()
            assert err < 2e-2 * ref.abs().max().item(), (name, pol, err)
        fns = [lambda: F.linear(a, b)] + [lambda p=p: C.gemm_ps_diag(a, b, c, 0, p) for p in range(4)] + \
              [lambda: C.gemm_ps_diag(a, b, c, 7, 0)] + \
              [lambda sg=sg: C.gemm_ps_diag(a, b, c, 0, 0, None, 0, sg) for sg in (1, 2)]
        t = timeit(fns, rounds=7, it=10)
        fl = 2.0 * M * n * k
        print(f"{name:7s} N={n:5d} K={k:5d}  library {t[0]:7.1f} us ({fl / t[0] / 1e6:5.0f} TF)  plain {t[1]:7.1f}  "
              f"nt {t[2]:7.1f}  sc1 {t[3]:7.1f}  sc0sc1 {t[4]:7.1f}  no-store {t[5]:7.1f}  "
              f"4-phase stagger x1 {t[6]:7.1f}  x2 {t[7]:7.1f}", flush=True)
        for pol, nm in ((0, "plain"), (2, "sc1")):
            print(f"   stamps {nm:8s} {stamps_summary(a, b, c, 0, pol)}", flush=True)
        print(f"   stamps stagger1 {stamps_summary(a, b, c, 0, 0, 1)}", flush=True)
        print(f"   stamps stagger2 {stamps_summary(a, b, c, 0, 0, 2)}", flush=True)
        print(f"   stamps no-store {stamps_summary(a, b, c, 7, 0)}", flush=True)


if __name__ == "__main__":
    main()
