"""fc2 input-gradient GEMM with hipBLASLt's DGELU epilogue vs the unfused path, GPT-2-small MLP
shape (65536 x 768 x 3072): numerics of the fused d(GELU) against tanh- and erf-GELU
derivatives, and times of every piece (TunableOp-selected GEMMs for the unfused path)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

K = native()
dev, bf = "cuda", torch.bfloat16
M, C, Fd = 65536, 768, 3072
torch.manual_seed(0)
h = torch.randn(M, C, device=dev).to(bf)
w1 = (torch.randn(Fd, C, device=dev) * 0.05).to(bf)
b1 = (torch.randn(Fd, device=dev) * 0.5).to(bf)
w2 = (torch.randn(C, Fd, device=dev) * 0.02).to(bf)
dy = torch.randn(M, C, device=dev).to(bf)


def bench(fn, it=15):
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


pre = F.linear(h, w1, b1)  # biased pre-activation
dpre = torch.empty_like(pre)
ok = K.lt_matmul(dy, w2, dpre, False, False, K.LT_EPI_DGELU, None, pre)
print("DGELU ok:", ok, flush=True)
dact = (dy.float() @ w2.float())
pf = pre.float()
for name, approx in (("tanh", "tanh"), ("erf", "none")):
    x = pf.clone().requires_grad_()
    F.gelu(x, approximate=approx).backward(dact)
    r = x.grad
    print(f"  DGELU vs {name}-GELU': rel {float((dpre.float() - r).norm() / r.norm()):.3e} "
          f"max {(dpre.float() - r).abs().max().item():.3e}", flush=True)
# GELU epilogue forward numerics (for completeness)
act = torch.empty_like(pre)
if K.lt_matmul(h, w1, act, False, True, 36, b1, None):
    for name, approx in (("tanh", "tanh"), ("erf", "none")):
        r = F.gelu(pf, approximate=approx)
        print(f"  GELU_BIAS vs {name}: rel {float((act.float() - r).norm() / r.norm()):.3e}", flush=True)
t = {}
t["dgrad mm (TunableOp)"] = bench(lambda: dy.mm(w2))
o = torch.empty_like(pre)
t["dgrad lt DEFAULT"] = bench(lambda: K.lt_matmul(dy, w2, o, False, False, K.LT_EPI_DEFAULT))
t["dgrad lt DGELU"] = bench(lambda: K.lt_matmul(dy, w2, dpre, False, False, K.LT_EPI_DGELU, None, pre))
pre_nb = F.linear(h, w1)
da = dy.mm(w2)
t["bias_gelu_bwd (HIP, incl. bias grad)"] = bench(lambda: K.bias_gelu_bwd(pre_nb, b1, da))
t["gelu_bwd (HIP)"] = bench(lambda: K.gelu_bwd(pre, da))
t["colsum_bf16 of dpre"] = bench(lambda: K.colsum_bf16(dpre))
t["fwd F.linear no bias"] = bench(lambda: F.linear(h, w1))
t["fwd F.linear + bias"] = bench(lambda: F.linear(h, w1, b1))
t["fwd bias_gelu_fwd (HIP)"] = bench(lambda: K.bias_gelu_fwd(pre_nb, b1))
t["fwd gelu_fwd (HIP)"] = bench(lambda: K.gelu_fwd(pre))
for k, v in t.items():
    print(f"{k:40s} {v:8.1f} us", flush=True)
