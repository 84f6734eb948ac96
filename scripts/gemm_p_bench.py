"""Persistent role-split GEMM (csrc/kernels/gemm_persistent.hip, `gemm_p`) vs the library GEMM and
the tiled gemm_nt at the GPT-2-small bench shapes (B*T = 65536 tokens): correctness against fp32
first (every epilogue, both layouts, a half tile at the right edge), then time per call on random
operands (median of interleaved rounds in one process).

    python scripts/gemm_p_bench.py [--quick]
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
    cases = [(256, 256, 192), (512, 768, 256), (1024, 512, 768), (2048, 3072, 768), (768, 384, 320),
             (4096, 2304, 768), (256 * 300, 768, 768)]
    for (m, n, k) in cases:
        a = torch.randn(m, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.05
        bias = torch.randn(n, device=dev, dtype=bf) * 0.1
        ref = a.float() @ b.float().t()
        for layout in (0, 1):
            if not C.gemm_p_supported(m, n, k, layout):
                continue
            bb = b if layout == 0 else b.t().contiguous()
            for epi in range(4):
                c = torch.empty(m, n, device=dev, dtype=bf)
                c2 = torch.randn(m, n, device=dev, dtype=bf) if epi == 3 else torch.empty(m, n, device=dev, dtype=bf)
                cs = torch.zeros(n, device=dev, dtype=torch.float32)
                pre_in = c2.clone()
                C.gemm_p(a, bb, c, c2, bias, cs, epi, layout)
                torch.cuda.synchronize()
                if epi == 0:
                    want = ref
                elif epi == 1:
                    want = ref + bias.float()
                elif epi == 2:
                    want = ref + bias.float()
                    g = F.gelu(want, approximate="tanh")
                    e2 = (c2.float() - g).abs().max().item()
                    assert e2 < 3e-2 * g.abs().max().item(), (m, n, k, layout, "gelu", e2)
                else:
                    x = pre_in.float().requires_grad_()
                    F.gelu(x, approximate="tanh").backward(ref)
                    want = x.grad
                    ecs = (cs - c.float().sum(0)).abs().max().item()
                    assert ecs < 1e-2 * c.float().sum(0).abs().max().item() + 1e-3, (m, n, k, layout, "colsum", ecs)
                err = (c.float() - want).abs().max().item()
                tol = 2e-2 * want.abs().max().item()
                assert err < tol, (m, n, k, layout, epi, err, tol)
            print(f"ok  M={m} N={n} K={k} layout={layout} epilogues 0-3", flush=True)
    # half tile at the right edge (N % 256 == 128, e.g. the padded GPT-2 vocabulary)
    for (m, n, k) in [(512, 384, 256), (1024, 1408, 768)]:
        a = torch.randn(m, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.05
        c = torch.full((m, n + 64), 7.0, device=dev, dtype=bf)[:, :n]
        C.gemm_p(a, b, c, None, None, None, 0, 0)
        torch.cuda.synchronize()
        ref = a.float() @ b.float().t()
        err = (c.float() - ref).abs().max().item()
        assert err < 2e-2 * ref.abs().max().item(), (m, n, k, "edge", err)
        print(f"ok  M={m} N={n} K={k} half edge tile", flush=True)


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


def check4():
    for (m, n, k) in [(256, 256, 128), (512, 768, 256), (2048, 3072, 768), (4096, 2304, 768)]:
        a = torch.randn(m, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.05
        c = torch.empty(m, n, device=dev, dtype=bf)
        C.gemm4(a, b, c)
        torch.cuda.synchronize()
        ref = a.float() @ b.float().t()
        err = (c.float() - ref).abs().max().item()
        assert err < 2e-2 * ref.abs().max().item(), (m, n, k, "gemm4", err)
        print(f"ok  gemm4 M={m} N={n} K={k}", flush=True)


def main():
    check4()
    if "--gemm4" in sys.argv:
        for name, n, k in [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072)]:
            a = torch.randn(M, k, device=dev, dtype=bf)
            b = torch.randn(n, k, device=dev, dtype=bf) * 0.02
            c = torch.empty(M, n, device=dev, dtype=bf)
            fl = 2.0 * M * n * k
            t_lib, t_nt, t_4 = timeit([lambda: F.linear(a, b), lambda: C.gemm_nt(a, b, c), lambda: C.gemm4(a, b, c)])
            print(f"{name:7s} N={n:5d} K={k:5d}  library {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)  gemm_nt {t_nt:7.1f} "
                  f"({fl / t_nt / 1e6:5.0f})  gemm4 {t_4:7.1f} ({fl / t_4 / 1e6:5.0f} TF)", flush=True)
        for n in (4096, 8192):
            a = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
            b = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
            c = torch.empty(n, n, device=dev, dtype=bf)
            fl = 2.0 * n ** 3
            t_lib, t_nt, t_4 = timeit([lambda: F.linear(a, b), lambda: C.gemm_nt(a, b, c), lambda: C.gemm4(a, b, c)])
            print(f"{n}^3  library {fl / t_lib / 1e6:5.0f} TF  gemm_nt {fl / t_nt / 1e6:5.0f} TF  gemm4 {fl / t_4 / 1e6:5.0f} TF",
                  flush=True)
        return
    check()
    quick = "--quick" in sys.argv
    shapes = [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072)]
    tl = tn = tp = 0.0
    print("forward (NT, x W^T)", flush=True)
    for name, n, k in shapes:
        a = torch.randn(M, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        c = torch.empty(M, n, device=dev, dtype=bf)
        fl = 2.0 * M * n * k
        t_lib, t_nt, t_p = timeit([lambda: F.linear(a, b), lambda: C.gemm_nt(a, b, c), lambda: C.gemm_p(a, b, c)])
        tl, tn, tp = tl + t_lib, tn + t_nt, tp + t_p
        print(f"{name:7s} N={n:5d} K={k:5d}  library {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)  gemm_nt {t_nt:7.1f} "
              f"({fl / t_nt / 1e6:5.0f})  gemm_p {t_p:7.1f} ({fl / t_p / 1e6:5.0f} TF)", flush=True)
        del a, b, c
    print("input gradient (NN, dY W)", flush=True)
    for name, n_out, k_in in [("dg_qkv", 2304, 768), ("dg_proj", 768, 768), ("dg_fc", 3072, 768), ("dg_fc2", 768, 3072)]:
        dy = torch.randn(M, n_out, device=dev, dtype=bf)
        w = torch.randn(n_out, k_in, device=dev, dtype=bf) * 0.02
        c = torch.empty(M, k_in, device=dev, dtype=bf)
        fl = 2.0 * M * n_out * k_in
        wt = w.t().contiguous()
        t_lib, t_nt, t_p = timeit([lambda: torch.mm(dy, w), lambda: C.gemm_nt(dy, wt, c), lambda: C.gemm_p(dy, w, c, layout=1)])
        tl, tn, tp = tl + t_lib, tn + t_nt, tp + t_p
        print(f"{name:7s} N={k_in:5d} K={n_out:5d}  library {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)  gemm_nt(W^T) {t_nt:7.1f} "
              f"({fl / t_nt / 1e6:5.0f})  gemm_p NN {t_p:7.1f} ({fl / t_p / 1e6:5.0f} TF)", flush=True)
        del dy, w, c, wt
    print(f"total (8 shapes) library {tl:.0f} us, gemm_nt {tn:.0f} us, gemm_p {tp:.0f} us", flush=True)
    # fused epilogues
    a = torch.randn(M, 768, device=dev, dtype=bf)
    w = torch.randn(3072, 768, device=dev, dtype=bf) * 0.02
    bias = torch.zeros(3072, device=dev, dtype=bf)
    pre = torch.empty(M, 3072, device=dev, dtype=bf)
    act = torch.empty_like(pre)
    t_lib, t_fused = timeit([lambda: C.bias_gelu_fwd(F.linear(a, w), bias) if hasattr(C, "bias_gelu_fwd") else F.gelu(F.linear(a, w, bias), approximate="tanh"),
                             lambda: C.gemm_p(a, w, pre, act, bias, None, 2)])
    print(f"fc + bias + gelu: library GEMM + pass {t_lib:7.1f} us   gemm_p fused {t_fused:7.1f} us", flush=True)
    dy = torch.randn(M, 768, device=dev, dtype=bf)
    w2 = torch.randn(768, 3072, device=dev, dtype=bf) * 0.02
    cs = torch.zeros(3072, device=dev, dtype=torch.float32)
    dpre = torch.empty_like(pre)
    t_f = timeit([lambda: C.gemm_p(dy, w2, dpre, pre, None, cs, 3, 1)])[0]
    t_l = timeit([lambda: torch.mm(dy, w2)])[0]
    print(f"fc2 dgrad + dgelu + bias grad: gemm_p NN fused {t_f:7.1f} us (library dgrad alone {t_l:7.1f} us)", flush=True)
    if quick:
        return
    # LM head (N = 50304 = 196.5 tiles of 256) and its input gradient (K = 50304)
    x = torch.randn(M, 768, device=dev, dtype=bf)
    wte = torch.randn(50304, 768, device=dev, dtype=bf) * 0.02
    logits = torch.empty(M, 50304, device=dev, dtype=bf)
    fl = 2.0 * M * 50304 * 768
    t_lib, t_p = timeit([lambda: F.linear(x, wte), lambda: C.gemm_p(x, wte, logits)], rounds=3, it=3)
    print(f"lm_head N=50304 K=768  library {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)  gemm_p {t_p:7.1f} ({fl / t_p / 1e6:5.0f} TF)", flush=True)
    dx = torch.empty(M, 768, device=dev, dtype=bf)
    t_lib, t_p = timeit([lambda: torch.mm(logits, wte), lambda: C.gemm_p(logits, wte, dx, layout=1)], rounds=3, it=3)
    print(f"dg_lm   N=768 K=50304  library {t_lib:7.1f} us ({fl / t_lib / 1e6:5.0f} TF)  gemm_p NN {t_p:7.1f} ({fl / t_p / 1e6:5.0f} TF)", flush=True)
    for n in (4096, 8192):
        a = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
        b = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
        c = torch.empty(n, n, device=dev, dtype=bf)
        fl = 2.0 * n ** 3
        t_lib, t_nt, t_p = timeit([lambda: F.linear(a, b), lambda: C.gemm_nt(a, b, c), lambda: C.gemm_p(a, b, c)])
        print(f"{n}^3  library {fl / t_lib / 1e6:5.0f} TF  gemm_nt {fl / t_nt / 1e6:5.0f} TF  gemm_p {fl / t_p / 1e6:5.0f} TF", flush=True)


if __name__ == "__main__":
    main()
