"""gemm_wg against the library weight gradient at the Llama-3-8B shapes of config 5 (B=2 x T=2048 = 4096 tokens per
step): dW[N, K] = dY[4096, N]^T X[4096, K] for q / o (4096 x 4096), k / v (1024 x 4096), gate / up (14336 x 4096)
and down (4096 x 14336). The library path is what ops.linear.wgrad runs for them today (gemm_wg_ok refuses outputs
of more than 128 tiles); gemm_wg runs with its own split count. Median of 5 interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402

from distributedvolunteercomputing_amd import config  # noqa: E402
from distributedvolunteercomputing_amd.ops import native  # noqa: E402
import importlib  # noqa: E402

L = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")
C = native()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
shapes = {"q/o": (4096, 4096), "k/v": (1024, 4096), "gate/up": (14336, 4096), "down": (4096, 14336)}
torch.manual_seed(0)
cases = []
for name, (N, K) in shapes.items():
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)

    def lib(dy=dy, x=x, g=g):
        with config.override(gemm_wgrad="lib"):
            L.wgrad(dy, x, out=g, accumulate=True)
    cases.append((name, N, K, "library", lib))
    if C.gemm_wg_supported(N, K, M):
        cases.append((name, N, K, "gemm_wg", lambda dy=dy, x=x, g=g: C.gemm_wg(dy, x, g, True)))
        ref = (dy.float().t() @ x.float())
        o = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        C.gemm_wg(dy, x, o, False)
        torch.cuda.synchronize()
        print(f"{name}: gemm_wg rel err {((o.float() - ref).norm() / ref.norm()).item():.2e}, "
              f"splits {C.gemm_wg_splits(N, K, M) if hasattr(C, 'gemm_wg_splits') else '?'}", flush=True)


def tm(fn, it=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


res = {}
for rnd in range(5):
    for name, N, K, kind, fn in cases:
        res.setdefault((name, kind), []).append(tm(fn))
for name, N, K, kind, _ in cases:
    t = sorted(res[(name, kind)])[2]
    print(f"wgrad {name:8s} {kind:8s} {t:9.1f} us  {2.0 * M * N * K / t / 1e6:6.0f} TF", flush=True)
