"""gemm_f (csrc/kernels/gemm_f.hip) against the library forward GEMM at the GPT-2 step's shapes (M = 64 x 1024
tokens): Y[M, N] = X[M, K] W[N, K]^T + b for qkv (2304 x 768), attention projection (768 x 768), fc (3072 x 768) and
fc2 (768 x 3072), plus the square 4096^3 (also Llama-3-8B's q/o forward at 4096 tokens). Relative error
against an fp32 product first, then the median of 5 interleaved rounds of 5 launches each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
shapes = {"qkv": (M, 2304, 768), "proj": (M, 768, 768), "fc": (M, 3072, 768), "fc2": (M, 768, 3072),
          "sq4096": (4096, 4096, 4096), "lm_head": (M, 50304, 768)}
WAVES = [int(w) for w in os.environ.get("GEMM_F_WAVES", "4,8").split(",")]
only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else None  # e.g. "sq4096,lm_dgrad" (counter passes)
torch.manual_seed(0)
cases = []
for name, (m, N, K) in shapes.items():
    if only and name not in only:
        continue
    x = torch.randn(m, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
    y = torch.empty(m, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
    cases.append((name, m, N, K, "library", lambda x=x, w=w, bias=bias: F.linear(x, w, bias)))
    if C.gemm_f_supported(m, N, K):
        C.gemm_f(x, w, y, bias)
        ref = (x.float() @ w.float().t()).add_(bias.float())
        torch.cuda.synchronize()
        err = ((y.float() - ref).norm() / ref.norm()).item()
        print(f"{name}: gemm_f rel err {err:.2e}", flush=True)
        if not err < 1e-2:
            sys.exit(f"{name}: gemm_f wrong")
        for wv in WAVES:
            C.gemm_f(x, w, y, bias, wv)
            torch.cuda.synchronize()
            err = ((y.float() - ref).norm() / ref.norm()).item()
            if not err < 1e-2:
                sys.exit(f"{name}: gemm_f waves {wv} wrong ({err:.2e})")
            print(f"{name}: gemm_f waves {wv} rel err {err:.2e}", flush=True)
            cases.append((name, m, N, K, f"gemm_f{wv}", lambda x=x, w=w, y=y, bias=bias, wv=wv: C.gemm_f(x, w, y, bias, wv)))


def tm(fn, it=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


# the LM head's input gradient dX[M, 768] = dL[M, 50304] W[50304, 768]: the library's NN product against gemm_f
# with the transposed tied weight (a 77 MB copy per step)
if not only or "lm_dgrad" in only:
    dl = torch.randn(M, 50304, device="cuda", dtype=torch.bfloat16) * 0.01
    wte = torch.randn(50304, 768, device="cuda", dtype=torch.bfloat16) * 0.02
    wt = wte.t().contiguous()
    dx = torch.empty(M, 768, device="cuda", dtype=torch.bfloat16)
    C.gemm_f(dl, wt, dx)
    ref = dl.float() @ wte.float()
    torch.cuda.synchronize()
    print(f"lm_dgrad: gemm_f rel err {((dx.float() - ref).norm() / ref.norm()).item():.2e}", flush=True)
    del ref
    cases.append(("lm_dgrad", M, 768, 50304, "library", lambda: torch.mm(dl, wte)))
    for wv in WAVES:
        cases.append(("lm_dgrad", M, 768, 50304, f"gemm_f{wv}", lambda wv=wv: C.gemm_f(dl, wt, dx, None, wv)))
    cases.append(("lm_dgrad", M, 768, 50304, "gemm_f8+T", lambda: C.gemm_f(dl, wte.t().contiguous(), dx, None, 8)))

res = {}
for rnd in range(5):
    for name, m, N, K, kind, fn in cases:
        res.setdefault((name, kind), []).append(tm(fn))
for name, m, N, K, kind, _ in cases:
    t = sorted(res[(name, kind)])[2]
    print(f"fwd {name:7s} {kind:8s} {t:9.1f} us  {2.0 * m * N * K / t / 1e6:6.0f} TF", flush=True)
