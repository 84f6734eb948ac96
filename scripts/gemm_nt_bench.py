"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) vs the library GEMM at the GPT-2-small bench
shapes (B*T = 65536 tokens): correctness against fp32 and time per call, random operands.

    python scripts/gemm_nt_bench.py
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
SHAPES = [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072),
          ("dg_fc2", 3072, 768), ("dg_fc", 768, 3072), ("dg_qkv", 768, 2304)]


def bench(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def check():
    torch.manual_seed(0)
    for (m, n, k) in [(256, 256, 128), (512, 768, 192), (1024, 512, 768), (2048, 3072, 768)]:
        a = torch.randn(m, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.05
        bias = torch.randn(n, device=dev, dtype=bf) * 0.1
        ref = a.float() @ b.float().t()
        for epi in range(4):
            c = torch.empty(m, n, device=dev, dtype=bf)
            c2 = torch.randn(m, n, device=dev, dtype=bf) if epi == 3 else torch.empty(m, n, device=dev, dtype=bf)
            cs = torch.zeros(n, device=dev, dtype=torch.float32)
            pre_in = c2.clone()
            C.gemm_nt(a, b, c, c2, bias, cs, epi)
            torch.cuda.synchronize()
            if epi == 0:
                want = ref
            elif epi == 1:
                want = ref + bias.float()
            elif epi == 2:
                want = ref + bias.float()
                g = F.gelu(want, approximate="tanh")
                e2 = (c2.float() - g).abs().max().item()
                assert e2 < 3e-2 * g.abs().max().item(), (m, n, k, "gelu", e2)
            else:
                x = pre_in.float().requires_grad_()
                F.gelu(x, approximate="tanh").backward(ref)
                want = x.grad
                ecs = (cs - c.float().sum(0)).abs().max().item()
                assert ecs < 1e-2 * c.float().sum(0).abs().max().item() + 1e-3, (m, n, k, "colsum", ecs)
            err = (c.float() - want).abs().max().item()
            tol = 2e-2 * want.abs().max().item()
            assert err < tol, (m, n, k, epi, err, tol)
            print(f"ok  M={m} N={n} K={k} epi={epi}  max err {err:.3e} (tol {tol:.3e})", flush=True)


def main():
    check()
    tot_lib = tot_mine = 0.0
    for name, n, k in SHAPES:
        a = torch.randn(M, k, device=dev, dtype=bf)
        b = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        c = torch.empty(M, n, device=dev, dtype=bf)
        fl = 2.0 * M * n * k
        t_lib = bench(lambda: F.linear(a, b))
        t_mine = bench(lambda: C.gemm_nt(a, b, c))
        tot_lib += t_lib
        tot_mine += t_mine
        print(f"{name:7s} N={n:5d} K={k:5d}  library {t_lib:8.1f} us ({fl / t_lib / 1e6:6.0f} TF)   "
              f"gemm_nt {t_mine:8.1f} us ({fl / t_mine / 1e6:6.0f} TF)", flush=True)
        del a, b, c
    print(f"total library {tot_lib:.0f} us, gemm_nt {tot_mine:.0f} us", flush=True)
    # fused MLP epilogues against library GEMM + separate elementwise passes
    a = torch.randn(M, 768, device=dev, dtype=bf)
    w = torch.randn(3072, 768, device=dev, dtype=bf) * 0.02
    bias = torch.zeros(3072, device=dev, dtype=bf)
    pre = torch.empty(M, 3072, device=dev, dtype=bf)
    act = torch.empty_like(pre)
    t = bench(lambda: C.gemm_nt(a, w, pre, act, bias, None, 2))
    print(f"fc + bias + gelu (fused epilogue) {t:8.1f} us", flush=True)
    dy = torch.randn(M, 768, device=dev, dtype=bf)
    w2t = torch.randn(3072, 768, device=dev, dtype=bf) * 0.02
    cs = torch.zeros(3072, device=dev, dtype=torch.float32)
    dpre = torch.empty_like(pre)
    t = bench(lambda: C.gemm_nt(dy, w2t, dpre, pre, None, cs, 3))
    print(f"fc2 dgrad + dgelu + bias grad (fused epilogue) {t:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
