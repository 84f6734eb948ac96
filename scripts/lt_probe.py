"""hipBLASLt epilogue probe at the GPT-2-small MLP shape (B*T = 65536 tokens, C = 768, F = 3072).

Checks the fused epilogues of csrc/bindings_lt.cpp against fp32 torch references and times them
against the unfused path (library GEMM + HIP bias/GELU kernels) in one process:
  fc  forward : GELU_AUX_BIAS  vs  F.linear + bias_gelu_fwd
  fc2 dgrad   : DGELU_BGRAD    vs  dy.mm(W2) + bias_gelu_bwd (incl. its bias-grad column sums)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
C, Fd = 768, 3072
dev, bf = "cuda", torch.bfloat16
K = native()
torch.manual_seed(0)
h = torch.randn(M, C, device=dev).to(bf)
w1 = (torch.randn(Fd, C, device=dev) * 0.02).to(bf)
b1 = (torch.randn(Fd, device=dev) * 0.5).to(bf)
w2 = (torch.randn(C, Fd, device=dev) * 0.02).to(bf)
dy = torch.randn(M, C, device=dev).to(bf)


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


def rel(a, r):
    return float((a.float() - r).norm() / r.norm())


# ---------------- fc forward: numerics
pre = torch.empty(M, Fd, device=dev, dtype=bf)
act = torch.empty_like(pre)
ok = K.lt_matmul(h, w1, act, False, True, K.LT_EPI_GELU_AUX_BIAS, b1, pre)
print("GELU_AUX_BIAS supported:", ok, flush=True)
if ok:
    pre_ref = h.float() @ w1.float().t() + b1.float()
    print(f"  pre rel err {rel(pre, pre_ref):.2e}  act vs tanh-gelu {rel(act, F.gelu(pre_ref, approximate='tanh')):.2e}"
          f"  act vs erf-gelu {rel(act, F.gelu(pre_ref)):.2e}", flush=True)
    # tanh vs erf on the kernel's own pre-activation: the discriminating comparison
    pf = pre.float()
    print(f"  max|act - tanh(pre)| {(act.float() - F.gelu(pf, approximate='tanh')).abs().max().item():.3e}"
          f"  max|act - erf(pre)| {(act.float() - F.gelu(pf)).abs().max().item():.3e}", flush=True)
    t_f = bench(lambda: K.lt_matmul(h, w1, act, False, True, K.LT_EPI_GELU_AUX_BIAS, b1, pre))
    t_u = bench(lambda: K.bias_gelu_fwd(F.linear(h, w1), b1))
    t_g = bench(lambda: F.linear(h, w1))
    print(f"  fused {t_f:8.1f} us   unfused (tuned GEMM + HIP bias_gelu) {t_u:8.1f} us   GEMM alone {t_g:8.1f} us",
          flush=True)

# ---------------- fc2 dgrad with DGELU + bias grad
dpre = torch.empty(M, Fd, device=dev, dtype=bf)
db = torch.empty(Fd, device=dev, dtype=bf)
ok2 = K.lt_matmul(dy, w2, dpre, False, False, K.LT_EPI_DGELU_BGRAD, db, pre)
print("DGELU_BGRAD supported:", ok2, flush=True)
if ok2:
    pf = pre.float().requires_grad_()
    g = F.gelu(pf, approximate="tanh")
    g.backward(dy.float() @ w2.float())
    print(f"  dpre rel err {rel(dpre, pf.grad):.2e}   db rel err {rel(db, pf.grad.sum(0)):.2e}", flush=True)
    t_f = bench(lambda: K.lt_matmul(dy, w2, dpre, False, False, K.LT_EPI_DGELU_BGRAD, db, pre))
    # unfused: dgrad GEMM then bias_gelu_bwd (x there is the pre-activation WITHOUT bias)
    pre_nb = (pre.float() - b1.float()).to(bf)
    t_u = bench(lambda: K.bias_gelu_bwd(pre_nb, b1, dy.mm(w2)))
    t_g = bench(lambda: dy.mm(w2))
    print(f"  fused {t_f:8.1f} us   unfused (tuned GEMM + HIP bias_gelu_bwd) {t_u:8.1f} us   GEMM alone {t_g:8.1f} us",
          flush=True)

dflt = torch.empty(M, Fd, device=dev, dtype=bf)
okd = K.lt_matmul(h, w1, dflt, False, True, K.LT_EPI_DEFAULT)
if okd:
    t = bench(lambda: K.lt_matmul(h, w1, dflt, False, True, K.LT_EPI_DEFAULT))
    print(f"lt DEFAULT fc fwd {t:8.1f} us (rel err vs F.linear {rel(dflt, F.linear(h, w1).float()):.1e})", flush=True)
print({k: round(v * 1e3, 1) for k, v in K.lt_tuned().items()})
