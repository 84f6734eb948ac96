"""Every GEMM of one GPT-2-small bench step (B=64 x T=1024, d=768) timed as the model issues it, and
the weight-gradient alternatives: which shapes the step GEMM time is made of, and where the library
is weakest. Median of interleaved rounds, TunableOp results loaded as in bench.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

TUNED = enable_tuned_gemms(0)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedvolunteercomputing_amd import config  # noqa: E402
import importlib  # noqa: E402

L = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")  # (ops.linear is also a function)
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
M, d = 65536, 768
shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "lm": (50304, 768)}
C = native()
torch.manual_seed(0)
cases = []
for name, (N, K) in shapes.items():
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    cases.append((f"fwd   {name}", fl, lambda x=x, w=w: F.linear(x, w)))
    cases.append((f"dgrad {name}", fl, lambda dy=dy, w=w: torch.mm(dy, w)))
    if C.gemm_ps_supported(M, K, N, 0):  # dX[M, K] = dY W on W^T (ops/linear.py dgrad_ps_ok)
        wt = L.transpose_weight(w)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        cases.append((f"dgrad {name} gemm_ps", fl, lambda dy=dy, wt=wt, dx=dx: C.gemm_ps(dy, wt, dx)))
    cases.append((f"wgrad {name} default", fl, lambda dy=dy, x=x, gw=gw: L.wgrad(dy, x, out=gw, accumulate=True)))

    def libw(dy=dy, x=x, gw=gw):
        with config.override(gemm_wgrad="lib"):
            L.wgrad(dy, x, out=gw, accumulate=True)
    cases.append((f"wgrad {name} library(S={L._splits(M, N, K)})", fl, libw))
    cases.append((f"wgrad {name} one GEMM", fl, lambda dy=dy, x=x, gw=gw: gw.addmm_(dy.t(), x)))
    for S in (4, 8, 32):
        if M % S == 0:
            def f(dy=dy, x=x, gw=gw, S=S, N=N, K=K):
                part = torch.bmm(dy.view(S, M // S, N).transpose(1, 2), x.view(S, M // S, K))
                C.splitk_reduce(part, gw, True)
            cases.append((f"wgrad {name} bmm S={S}", fl, f))
    if C.gemm_wg_supported(N, K, M):
        cases.append((f"wgrad {name} gemm_wg", fl, lambda dy=dy, x=x, gw=gw: C.gemm_wg(dy, x, gw, True)))

ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
for _, _, fn in cases:
    fn()
torch.cuda.synchronize()
res = {c[0]: [] for c in cases}
for rnd in range(5):
    for name, fl, fn in cases:
        e0, e1 = ev(), ev()
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        e1.synchronize()
        res[name].append(e0.elapsed_time(e1) / 5 * 1e3)
print(f"tuned_gemms={TUNED}  M={M}", flush=True)
for name, fl, _ in cases:
    t = sorted(res[name])[len(res[name]) // 2]
    print(f"{name:34s} {t:9.1f} us  {fl / t / 1e6:7.0f} TF", flush=True)
