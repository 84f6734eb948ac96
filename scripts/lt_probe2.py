"""Which hipBLASLt epilogues have algorithms at the GPT-2 MLP shape (bf16, this hipBLASLt build),
and the LM-head GEMM timed hot vs cold (L2/MALL flushed) against its in-step time."""
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
h = torch.randn(M, C, device=dev).to(bf)
w1 = (torch.randn(Fd, C, device=dev) * 0.02).to(bf)
w2 = (torch.randn(C, Fd, device=dev) * 0.02).to(bf)
dy = torch.randn(M, C, device=dev).to(bf)
out = torch.empty(M, Fd, device=dev, dtype=bf)
aux = torch.empty_like(out)
for btype in (torch.bfloat16, torch.float32):
    b = torch.zeros(Fd, device=dev, dtype=btype)
    for name, epi, hb, ha in [("GELU", 32, 0, 0), ("GELU_BIAS", 36, 1, 0), ("GELU_AUX", 160, 0, 1),
                              ("GELU_AUX_BIAS", 164, 1, 1), ("BIAS", 4, 1, 0), ("RELU_BIAS", 6, 1, 0)]:
        for ta, tb, lab in ((False, True, "fwd TN"),):
            try:
                ok = K.lt_matmul(h, w1, out, ta, tb, epi, b if hb else None, aux if ha else None)
            except Exception as e:  # noqa: BLE001
                ok = f"error {str(e)[:80]}"
            print(f"{lab} {name:14s} bias={str(btype)[6:]:8s} -> {ok}", flush=True)
    for name, epi, hb in [("DGELU", 192, 0), ("DGELU_BGRAD", 208, 1), ("BGRADB", 512, 0)]:
        try:
            ok = K.lt_matmul(dy, w2, out, False, False, epi, b if hb else None, aux if epi in (192, 208) else None)
        except Exception as e:  # noqa: BLE001
            ok = f"error {str(e)[:80]}"
        print(f"dgrad NN {name:12s} bias={str(btype)[6:]:8s} -> {ok}", flush=True)

flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
wte = (torch.randn(50304, C, device=dev) * 0.02).to(bf)


def bench(fn, cold, it=8):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(it):
        if cold:
            flush.fill_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


for tag, fn in [("lm fwd F.linear", lambda: F.linear(h, wte)), ("lm fwd mm", lambda: torch.mm(h, wte.t()))]:
    print(f"{tag:18s} hot {bench(fn, False):.3f} ms  cold {bench(fn, True):.3f} ms", flush=True)
logits = torch.randn(M, 50304, device=dev).to(bf)
print(f"lm dgrad hot {bench(lambda: logits.mm(wte), False):.3f} ms cold {bench(lambda: logits.mm(wte), True):.3f}",
      flush=True)
print(f"lm wgrad (t.mm) hot {bench(lambda: logits.t().mm(h), False):.3f} ms", flush=True)
S = 4
print(f"lm wgrad bmm split4 hot "
      f"{bench(lambda: torch.bmm(logits.view(S, M // S, -1).transpose(1, 2), h.view(S, M // S, C)), False):.3f} ms",
      flush=True)
