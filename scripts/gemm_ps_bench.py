"""Persistent store-overlapped GEMM (csrc/kernels/gemm_ps.hip, `gemm_ps`) vs the library GEMM and the
tiled gemm_nt at the GPT-2-small bench shapes (B*T = 65536 tokens): correctness against fp32 first
(every epilogue, one tile per workgroup and several, a reduced grid), then time per call on random
operands (median of interleaved rounds in one process).

    python scripts/gemm_ps_bench.py [--check-only]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
dev = "cuda"
bf = torch.bfloat16
M = int(os.environ.get("GEMM_M", "65536"))


def check():
    torch.manual_seed(0)
    cases = [(256, 256, 256, 0), (512, 768, 256, 0), (2048, 3072, 768, 0), (4096, 2304, 768, 0),
             (256 * 300, 768, 768, 0), (4096, 2304, 768, 16), (8192, 768, 3072, 40), (1024, 512, 1024, 8),
             (65536, 2304, 768, 0), (65536, 768, 3072, 0), (16384, 768, 768, 0)]
    for (m, n, k, cap) in cases:
        a = torch.randn(m, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.05
        bias = torch.randn(n, device=dev, dtype=bf) * 0.1
        ref = a.float() @ b.float().t()
        for epi in range(3):
            c = torch.full((m, n), float("nan"), device=dev, dtype=bf)
            c2 = torch.full((m, n), float("nan"), device=dev, dtype=bf)
            C.gemm_ps(a, b, c, c2, bias, None, epi, cap)
            torch.cuda.synchronize()
            want = ref if epi == 0 else ref + bias.float()
            err = (c.float() - want).abs().max().item()
            tol = 2e-2 * want.abs().max().item()
            assert err < tol, (m, n, k, cap, epi, err, tol)
            if epi == 2:
                g = F.gelu(want, approximate="tanh")
                e2 = (c2.float() - g).abs().max().item()
                assert e2 < 3e-2 * g.abs().max().item(), (m, n, k, cap, "gelu", e2)
        # DGELU: c = (a b^T) * gelu'(pre), colsum += column sums of c (fp32, before rounding)
        pre = torch.randn(m, n, device=dev, dtype=bf)
        c = torch.full((m, n), float("nan"), device=dev, dtype=bf)
        cs = torch.zeros(n, device=dev, dtype=torch.float32)
        C.gemm_ps(a, b, c, pre, None, cs, 4, cap)
        torch.cuda.synchronize()
        x = pre.float().requires_grad_()
        F.gelu(x, approximate="tanh").backward(ref.to(bf).float())
        want = x.grad
        err = (c.float() - want).abs().max().item()
        assert err < 2e-2 * want.abs().max().item(), (m, n, k, cap, "dgelu", err)
        ecs = (cs - want.sum(0)).abs().max().item()
        assert ecs < 1e-2 * want.sum(0).abs().max().item() + 1e-2, (m, n, k, cap, "colsum", ecs)
        print(f"ok  M={m} N={n} K={k} grid_cap={cap} epilogues 0-2, 4", flush=True)


def timeit(fns, rounds=5, it=10):
    """Interleaved rounds of each fn; returns the median per-call microseconds of each."""
    res = [[] for _ in fns]
    for f in fns:
        for _ in range(2):
            f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for i, f in enumerate(fns):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(it):
                f()
            e1.record()
            e1.synchronize()
            res[i].append(e0.elapsed_time(e1) * 1e3 / it)
    return [sorted(r)[len(r) // 2] for r in res]


def main():
    check()
    if "--check-only" in sys.argv:
        return
    tl = tn = 0.0
    shapes = [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072),
              ("dg_qkv", 768, 2304), ("dg_proj", 768, 768), ("dg_fc", 768, 3072), ("dg_fc2", 3072, 768)]
    for name, n, k in shapes:
        a = torch.randn(M, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        c = torch.empty(M, n, device=dev, dtype=bf)
        fl = 2.0 * M * n * k
        if name.startswith("dg_"):  # the library runs dY . W on the [K, N] weight; ours on W^T
            bt = b.t().contiguous()
            lib = lambda: torch.mm(a, bt)  # noqa: E731
        else:
            lib = lambda: F.linear(a, b)  # noqa: E731
        t_lib, t_ps = timeit([lib, lambda: C.gemm_ps(a, b, c)])
        tl, tn = tl + t_lib, tn + t_ps
        print(f"{name:7s} N={n:5d} K={k:5d}  library {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)  gemm_ps {t_ps:7.1f} "
              f"({fl / t_ps / 1e6:5.0f} TF)  ratio {t_lib / t_ps:5.3f}", flush=True)
    print(f"total (8 shapes) library {tl:.0f} us, gemm_ps {tn:.0f} us", flush=True)
    # fc + bias + GELU: library GEMM + the separate bias_gelu pass vs the fused epilogue
    a = torch.randn(M, 768, device=dev, dtype=bf)
    w = torch.randn(3072, 768, device=dev, dtype=bf) * 0.02
    bias = torch.randn(3072, device=dev, dtype=bf) * 0.02
    pre = torch.empty(M, 3072, device=dev, dtype=bf)
    act = torch.empty(M, 3072, device=dev, dtype=bf)
    from distributedvolunteercomputing_amd import ops
    t_lib, t_ps = timeit([lambda: ops.bias_gelu(F.linear(a, w), bias) if hasattr(ops, "bias_gelu") else None,
                          lambda: C.gemm_ps(a, w, pre, act, bias, epi=2)])
    print(f"fc + bias + gelu: library GEMM + pass {t_lib:7.1f} us   gemm_ps fused {t_ps:7.1f} us", flush=True)
    # fc2 input gradient + gelu' + bias grad: library dgrad + bias_gelu_bwd vs the fused DGELU epilogue
    dy = torch.randn(M, 768, device=dev, dtype=bf)
    w2 = torch.randn(768, 3072, device=dev, dtype=bf) * 0.02
    w2t = w2.t().contiguous()
    xpre = torch.randn(M, 3072, device=dev, dtype=bf)
    gb = torch.zeros(3072, device=dev, dtype=bf)
    cs = torch.zeros(3072, device=dev, dtype=torch.float32)
    dpre = torch.empty(M, 3072, device=dev, dtype=bf)
    t_lib, t_ps = timeit([lambda: C.bias_gelu_bwd(xpre, bias, torch.mm(dy, w2), gb),
                          lambda: C.gemm_ps(dy, w2t, dpre, xpre, None, cs, 4)])
    print(f"fc2 dgrad + dgelu + bias grad: library GEMM + pass {t_lib:7.1f} us   gemm_ps fused {t_ps:7.1f} us", flush=True)
    for n in (4096, 8192):
        a = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
        b = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
        c = torch.empty(n, n, device=dev, dtype=bf)
        fl = 2.0 * n ** 3
        t_lib, t_ps = timeit([lambda: F.linear(a, b), lambda: C.gemm_ps(a, b, c)])
        print(f"{n}^3  library {fl / t_lib / 1e6:5.0f} TF  gemm_ps {fl / t_ps / 1e6:5.0f} TF", flush=True)
    # grid sweep at the qkv shape (persistence: tiles per workgroup)
    a = torch.randn(M, 768, device=dev, dtype=bf)
    b = torch.randn(2304, 768, device=dev, dtype=bf) * 0.02
    c = torch.empty(M, 2304, device=dev, dtype=bf)
    caps = [256, 384, 512, 768, 1024]
    ts = timeit([lambda cc=cc: C.gemm_ps(a, b, c, grid_cap=cc) for cc in caps])
    print("qkv grid sweep: " + "  ".join(f"grid {cc}: {t:6.1f} us" for cc, t in zip(caps, ts)), flush=True)


if __name__ == "__main__":
    main()
