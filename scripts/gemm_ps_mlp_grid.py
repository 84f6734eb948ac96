"""Grid-cap sweep of the fused MLP epilogues on gemm_ps (5: fc forward bias + gelu/gelu', 6: fc2 input gradient x gelu' +
column sums) at the GPT-2 bench shape; cap 0 = one workgroup per CU (the default)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributedvolunteercomputing_amd.ops import native
C = native()
M, N, K = 65536, 3072, 768
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16); act = torch.empty_like(pre)
dy = torch.randn(M, 768, device="cuda", dtype=torch.bfloat16); w2t = torch.randn(N, 768, device="cuda", dtype=torch.bfloat16) * 0.03
out = torch.empty_like(pre); cs = torch.zeros(N, device="cuda")
def tm(fn, it=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); e0.record()
    for _ in range(it): fn()
    e1.record(); e1.synchronize(); return e0.elapsed_time(e1) / it * 1e3
for cap in [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "0,240,224,192,160,128,512").split(",")]:
    t5 = sorted(tm(lambda: C.gemm_ps(x, w, pre, act, b, None, 5, cap)) for _ in range(5))[2]
    t6 = sorted(tm(lambda: C.gemm_ps(dy, w2t, out, pre, None, cs, 6, cap)) for _ in range(5))[2]
    print(f"grid cap {cap:4d}: epi5 {t5:7.1f} us  epi6 {t6:7.1f} us", flush=True)
