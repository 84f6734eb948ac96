"""Tune the library GEMMs of the GPT-2-small bench step with PyTorch TunableOp on this GPU and merge the
winners into tuning/tunableop_gfx950.csv (utils/tuning.py loads that file read-only at run time).

Round 4: the committed file covered the forward / input-gradient GEMMs and single-GEMM weight gradients,
but not the token-split batched weight gradients the step actually runs (ops/linear.py wgrad: bmm of
S = 16 / 4 splits), which therefore ran the library's heuristic default. This tunes every GEMM of one
step by running the step's ops themselves: forward, input gradient, and the split weight gradients.

    python scripts/tune_gemms.py [out.csv]     (default: tuning/tunableop_gfx950.csv, merged in place)
"""
import importlib
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
RESULTS = os.path.join(ROOT, "tuning", "tunableop_gfx950.csv")
out_csv = sys.argv[1] if len(sys.argv) > 1 else RESULTS

work = tempfile.mkdtemp(prefix="vcx_tune_")
# start from the committed results: only shapes without an entry are tuned
shutil.copyfile(RESULTS, os.path.join(work, "results0.csv"))  # read at start: tuned shapes are skipped
os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(work, "results%d.csv")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "40")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS", "20")
os.environ["VCX_TUNABLEOP"] = "off"  # (enable_tuned_gemms would otherwise switch tuning off)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

L = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")

dev = torch.device("cuda", 0)
M = 65536
shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072), "lm": (50304, 768)}
torch.manual_seed(0)
for name, (N, K) in shapes.items():
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(2):
        F.linear(x, w)
        torch.mm(dy, w)
        L.wgrad(dy, x, out=gw, accumulate=True)  # the split (batched) weight gradient the step runs
    torch.cuda.synchronize()
    print(f"tuned {name}", flush=True)
    del x, w, dy, gw
    torch.cuda.empty_cache()
# the results file is only written when TunableOp shuts down: take the in-memory results instead
res = torch.cuda.tunable.get_results()
lines = open(RESULTS).read().splitlines() if os.path.exists(RESULTS) else []
have = {tuple(ln.split(",")[:2]) for ln in lines if ln and not ln.startswith("Validator")}
new = []
for r in res:
    op, params, kern, t = r[0], r[1], r[2], r[3]
    if (op, params) not in have:
        new.append(f"{op},{params},{kern},{t}")
print(f"{len(new)} new entries:", *new, sep="\n", flush=True)
with open(out_csv, "w") as f:
    f.write("\n".join(lines + new) + "\n")
print(f"wrote {out_csv}", flush=True)
