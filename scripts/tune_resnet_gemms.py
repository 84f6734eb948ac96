"""Tune the library GEMMs of the ResNet-50 config-3 step (its 1x1 convolutions run as NHWC GEMMs through
ops/linear.py: forward, input gradient and the token-split weight gradients) with PyTorch TunableOp and merge
the winners into a copy of tuning/tunableop_gfx950.csv (utils/tuning.py loads that file read-only at run time).
The committed table covered only the GPT-2 bench shapes; the ResNet shapes ran the library's heuristic.

    python scripts/tune_resnet_gemms.py out.csv
"""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
RESULTS = os.path.join(ROOT, "tuning", "tunableop_gfx950.csv")
out_csv = sys.argv[1]

work = tempfile.mkdtemp(prefix="vcx_tune_rn_")
shutil.copyfile(RESULTS, os.path.join(work, "results0.csv"))  # tuned shapes are skipped
os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
os.environ["PYTORCH_TUNABLEOP_FILENAME"] = os.path.join(work, "results%d.csv")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "40")
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS", "20")
os.environ["VCX_TUNABLEOP"] = "off"  # (enable_tuned_gemms would otherwise switch tuning off)

import torch  # noqa: E402

from distributedvolunteercomputing_amd.models.resnet import resnet50  # noqa: E402
from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer  # noqa: E402

dev = torch.device("cuda", 0)
m = resnet50().to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
tr = LocalSGDTrainer(m, LocalSGDConfig(H=4, lr=1e-3, weight_decay=0.0), device=dev)
x = torch.randn(128, 3, 224, 224, device=dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (128,), device=dev)
for i in range(2):
    tr.step(x, y)
    torch.cuda.synchronize()
    print(f"step {i} done", flush=True)
res = torch.cuda.tunable.get_results()
lines = open(RESULTS).read().splitlines()
have = {tuple(ln.split(",")[:2]) for ln in lines if ln and not ln.startswith("Validator")}
new = [f"{r[0]},{r[1]},{r[2]},{r[3]}" for r in res if (r[0], r[1]) not in have]
print(f"{len(new)} new entries:", *new, sep="\n", flush=True)
with open(out_csv, "w") as f:
    f.write("\n".join(lines + new) + "\n")
print(f"wrote {out_csv}", flush=True)
