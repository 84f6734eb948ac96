"""Weight-gradient token splits that are not powers of two, at the GPT-2-small bench shapes.

ops/linear.py wgrad runs dW = dY^T X as a batched library GEMM over S token chunks (S = 16, or 4 for
the LM head) plus the fp32 split-K reduce. S has been a power of two so the chunks tile M = 65536
exactly; the output is only 9-36 tiles of 256 x 256 per chunk, so S also sets how many workgroups
the GEMM has (S = 16: 144-576). Here S is free: S chunks of c = floor(M / S / 64) * 64 rows in the
batched GEMM, the leftover rows as one more bf16 partial (a single GEMM into part[S]), then the same
reduce -- the same precision as the power-of-two path (every partial is a bf16 GEMM output summed
in fp32). New shapes are tuned by TunableOp on their first call (as scripts/tune_gemms.py does).

    python scripts/wgrad_split_probe.py [results.csv] [--retune] [--splits name=S,S,...]

--retune drops the committed entries of the batched weight-gradient GEMMs before starting, so the
power-of-two splits are tuned again beside the new ones (same tuning budget for every candidate).
"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
args = sys.argv[1:]
RETUNE = "--retune" in args
OVR = {}
for a in args:
    if "=" in a and not a.startswith("--"):
        k, v = a.split("=")
        OVR[k] = [int(t) for t in v.split(",")]
pos = [a for a in args if not a.startswith("--") and "=" not in a]
out_csv = pos[0] if pos else None
os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
work = tempfile.mkdtemp(prefix="vcx_wsplit_")
with open(os.path.join(ROOT, "tuning", "tunableop_gfx950.csv")) as f:
    keep = [ln for ln in f if not (RETUNE and ln.startswith("GemmStridedBatchedTunableOp"))]
with open(os.path.join(work, "results0.csv"), "w") as f:
    f.writelines(keep)
os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(work, "results%d.csv")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "20")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS", "10")
os.environ["VCX_TUNABLEOP"] = "off"

import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
dev = torch.device("cuda", 0)
M = 65536
shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "lm": (50304, 768)}
SPLITS = {"lm": [1, 2, 3, 4, 6]}
SMALL = [8, 10, 12, 14, 16, 18, 20, 24, 28]
t_start = time.time()


def run(dy, x, out, S):
    N, K = dy.shape[1], x.shape[1]
    if S == 1:
        torch.mm(dy.t(), x, out=out)
        return
    c = (M // S) // 64 * 64
    main = S * c
    rem = M - main
    part = torch.empty(S + (1 if rem else 0), N, K, device=dev, dtype=torch.bfloat16)
    torch.bmm(dy[:main].view(S, c, N).transpose(1, 2), x[:main].view(S, c, K), out=part[:S])
    if rem:
        torch.mm(dy[main:].t(), x[main:], out=part[S])
    C.splitk_reduce(part, out, False)


torch.manual_seed(0)
for name, (N, K) in shapes.items():
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16) * 0.1
    out = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    ref = (dy.float().t() @ x.float()) if N * K < 16 * 1024 * 1024 else None
    splits = OVR.get(name, SPLITS.get(name, SMALL)) if not OVR or name in OVR else []
    if not splits:
        continue
    for S in splits:  # tune + check
        run(dy, x, out, S)
        torch.cuda.synchronize()
        if ref is not None:
            err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-2, (name, S, err)
        print(f"[{time.time() - t_start:6.1f}s] tuned {name} S={S}", flush=True)
    res = {S: [] for S in splits}
    for _ in range(5):  # interleaved rounds
        for S in splits:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run(dy, x, out, S)
            e1.record()
            e1.synchronize()
            res[S].append(e0.elapsed_time(e1) / 5 * 1e3)
    fl = 2.0 * M * N * K
    for S in splits:
        t = sorted(res[S])[2]
        c = (M // S) // 64 * 64 if S > 1 else M
        print(f"wgrad {name:4s} S={S:2d} (chunk {c}, rem {M - S * c if S > 1 else 0}): {t:8.1f} us  "
              f"{fl / t / 1e6:6.0f} TF", flush=True)
    del x, dy, out, ref
    torch.cuda.empty_cache()
if out_csv:
    with open(out_csv, "w") as f:
        for r in torch.cuda.tunable.get_results():
            f.write(",".join(str(v) for v in r[:4]) + "\n")
    print(f"wrote {out_csv}", flush=True)
