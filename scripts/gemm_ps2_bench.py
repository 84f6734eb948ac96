"""gemm_ps with two co-resident 4-wave workgroups per CU (waves=4, 256 x 128 tiles) vs the
one-workgroup-per-CU kernel (waves=8) vs the library at the GPT-2 shapes; correctness first.
stagger = how many ~8k-cycle sleeps the second half of the grid starts late."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.ops import native  # noqa: E402
from gemm_ps_bench import timeit  # noqa: E402

C = native()
dev, bf = "cuda", torch.bfloat16
torch.manual_seed(0)
for (m, n, k) in [(512, 256, 192), (2048, 384, 768), (4096, 2304, 768), (65536, 768, 768), (8192, 768, 3072)]:
    a = torch.randn(m, k, device=dev, dtype=bf)
    b = torch.randn(n, k, device=dev, dtype=bf) * 0.05
    bias = torch.randn(n, device=dev, dtype=bf) * 0.1
    ref = a.float() @ b.float().t()
    for epi in range(3):
        for st in (0, 2):
            c = torch.full((m, n), float("nan"), device=dev, dtype=bf)
            c2 = torch.full((m, n), float("nan"), device=dev, dtype=bf)
            C.gemm_ps(a, b, c, c2, bias, None, epi, 0, 4, st)
            torch.cuda.synchronize()
            want = ref if epi == 0 else ref + bias.float()
            err = (c.float() - want).abs().max().item()
            assert err < 2e-2 * want.abs().max().item(), (m, n, k, epi, st, err)
            if epi == 2:
                g = F.gelu(want, approximate="tanh")
                assert (c2.float() - g).abs().max().item() < 3e-2 * g.abs().max().item(), (m, n, k, "gelu")
    print(f"ok  waves=4 M={m} N={n} K={k}", flush=True)
M = 65536
for name, n, k in [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072), ("dg_qkv", 768, 2304),
                   ("dg_fc2", 3072, 768)]:
    a = torch.randn(M, k, device=dev, dtype=bf)
    b = torch.randn(n, k, device=dev, dtype=bf) * 0.02
    c = torch.empty(M, n, device=dev, dtype=bf)
    fns = [lambda: F.linear(a, b), lambda: C.gemm_ps(a, b, c), lambda: C.gemm_ps(a, b, c, waves=4),
           lambda: C.gemm_ps(a, b, c, waves=4, stagger=1), lambda: C.gemm_ps(a, b, c, waves=4, stagger=3),
           lambda: C.gemm_ps(a, b, c, epi=7, waves=4)]
    t = timeit(fns)
    print(f"{name:7s} N={n:5d} K={k:5d}  library {t[0]:6.1f}  ps8 {t[1]:6.1f}  ps4 {t[2]:6.1f}  ps4 st1 {t[3]:6.1f}  "
          f"ps4 st3 {t[4]:6.1f}  ps4 no-store {t[5]:6.1f} us", flush=True)
a = torch.randn(M, 768, device=dev, dtype=bf)
w = torch.randn(3072, 768, device=dev, dtype=bf) * 0.02
bias = torch.randn(3072, device=dev, dtype=bf) * 0.02
pre = torch.empty(M, 3072, device=dev, dtype=bf)
act = torch.empty_like(pre)
t = timeit([lambda: C.gemm_ps(a, w, pre, act, bias, epi=2), lambda: C.gemm_ps(a, w, pre, act, bias, epi=2, waves=4),
            lambda: C.gemm_ps(a, w, pre, act, bias, epi=2, waves=4, stagger=2)])
print(f"fc + bias + gelu fused: ps8 {t[0]:6.1f}  ps4 {t[1]:6.1f}  ps4 st2 {t[2]:6.1f} us", flush=True)
