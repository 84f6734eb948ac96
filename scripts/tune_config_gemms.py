"""Tune the library GEMMs of the BASELINE config steps with PyTorch TunableOp and merge the winners into a copy
of tuning/tunableop_gfx950.csv (utils/tuning.py loads that file read-only at run time): config 3 ResNet-50 (its
1x1 convolutions run as NHWC GEMMs through ops/linear.py: forward, input gradient and the token-split weight
gradients), config 4 GPT-2-medium, config 5 Llama-3-8B (the bench_configs.py shapes). The committed table first
covered only the GPT-2-small bench shapes; the others ran the library's heuristic.

    python scripts/tune_config_gemms.py out.csv [3,4,5]
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

import threading  # noqa: E402
import time  # noqa: E402

_t0 = time.time()


def _merged_lines():
    lines = open(RESULTS).read().splitlines()
    have = {tuple(ln.split(",")[:2]) for ln in lines if ln and not ln.startswith("Validator")}
    new = [f"{r[0]},{r[1]},{r[2]},{r[3]}" for r in torch.cuda.tunable.get_results() if (r[0], r[1]) not in have]
    return lines, new


def _heartbeat():  # tuning a big GEMM shape takes tens of seconds with no output of its own
    while True:
        time.sleep(30)
        try:  # the winners so far, so a run stopped at its time limit keeps what it tuned
            lines, new = _merged_lines()
            with open(out_csv + ".partial", "w") as f:
                f.write("\n".join(lines + new) + "\n")
        except Exception as e:  # noqa: BLE001
            new = [f"(partial write failed: {e})"]
        print(f"[tune] {time.time() - _t0:.0f} s, {len(new)} new entries so far", flush=True)


threading.Thread(target=_heartbeat, daemon=True).start()
dev = torch.device("cuda", 0)
configs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["3"]


def _steps(tr, x, y, tag):
    for i in range(2):
        tr.step(x, y)
        torch.cuda.synchronize()
        print(f"config {tag} step {i} done ({time.time() - _t0:.0f} s)", flush=True)


if "3" in configs:
    m = resnet50().to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=4, lr=1e-3, weight_decay=0.0), device=dev)
    x = torch.randn(128, 3, 224, 224, device=dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
    _steps(tr, x, torch.randint(0, 1000, (128,), device=dev), 3)
    del m, tr, x
    torch.cuda.empty_cache()
if "4" in configs:
    from distributedvolunteercomputing_amd.models.gpt2 import GPT2, GPT2Config

    cfg = GPT2Config.preset("gpt2-medium")
    m = GPT2(cfg).to(dev, torch.bfloat16)
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=4), device=dev)
    t = torch.randint(0, cfg.vocab_size, (32, 1025), device=dev)
    _steps(tr, t[:, :-1], t[:, 1:], 4)
    del m, tr, t
    torch.cuda.empty_cache()
if "5" in configs:
    from distributedvolunteercomputing_amd.models.llama import Llama, LlamaConfig
    from distributedvolunteercomputing_amd.parallel.zero import ShardedConfig, ShardedDPTrainer

    cfg = LlamaConfig.preset("llama3-8b")
    with torch.device("meta"):
        m = Llama(cfg, init=False)
    m = m.to_empty(device=dev).to(torch.bfloat16)
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0.0, 0.02) if p.dim() >= 2 else p.fill_(1.0)
    tr = ShardedDPTrainer(m, ShardedConfig(lr=1e-4), device=dev)
    t = torch.randint(0, cfg.vocab_size, (2, 2049), device=dev)
    _steps(tr, t[:, :-1], t[:, 1:], 5)
    del m, tr, t
    torch.cuda.empty_cache()
lines, new = _merged_lines()
print(f"{len(new)} new entries:", *new, sep="\n", flush=True)
with open(out_csv, "w") as f:
    f.write("\n".join(lines + new) + "\n")
print(f"wrote {out_csv}", flush=True)
