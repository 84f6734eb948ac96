"""Probe: LM head + fused cross-entropy at the GPT-2 bench shape, whole vs token-chunked.

Whole: logits [65536, 50304] = X W^T (6.6 GB written to HBM), xent_fused reads it and writes the
gradient in place. Chunked: the GEMM writes Mc rows at a time into ONE reused buffer (small
enough to stay in the 256 MB MALL), xent_fused runs on it, and the gradient chunk is copied into
the full dlogits buffer the backward GEMMs read. Prints ms per variant (median of 5)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
M, K, V, Vp = 65536, 768, 50257, 50304
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
w = (torch.randn(Vp, K, device=dev) * 0.02).to(torch.bfloat16)
tgt = torch.randint(0, V, (M,), device=dev)
nvalid = torch.tensor([float(M)], device=dev)
C = native()
full = torch.empty(M, Vp, device=dev, dtype=torch.bfloat16)


def whole():
    torch.matmul(x, w.t(), out=full)
    C.xent_fused(full, tgt, nvalid, V)


def chunked(mc, buf):
    for i in range(0, M, mc):
        torch.matmul(x[i:i + mc], w.t(), out=buf)
        C.xent_fused(buf, tgt[i:i + mc], nvalid, V)
        full[i:i + mc].copy_(buf)


def gemm_only(mc, buf):
    for i in range(0, M, mc):
        torch.matmul(x[i:i + mc], w.t(), out=buf)


def timeit(fn, *a):
    for _ in range(2):
        fn(*a)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(*a)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[2]


print(f"whole GEMM+xent            {timeit(whole):7.3f} ms", flush=True)
print(f"whole GEMM only            {timeit(gemm_only, M, full):7.3f} ms", flush=True)
for mc in (1024, 2048, 4096, 8192):
    buf = torch.empty(mc, Vp, device=dev, dtype=torch.bfloat16)
    print(f"chunk {mc:5d} GEMM+xent+copy {timeit(chunked, mc, buf):7.3f} ms   GEMM only {timeit(gemm_only, mc, buf):7.3f} ms",
          flush=True)
