"""Where the config-3 step (or, with argument gpt2, the bench.py GPT-2 step) (ResNet-50 local-SGD + top-k EF, B=128) launches torch copies and elementwise kernels:
torch.profiler over one step, every aten copy / elementwise op with its input shapes, device time and the deepest
stack frame inside this package. Diagnostic (prints a table)."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

enable_tuned_gemms(0)
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from distributedvolunteercomputing_amd.models.resnet import enable_conv_find, resnet50  # noqa: E402
from distributedvolunteercomputing_amd.parallel.compression import TopKCompressor  # noqa: E402
from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer  # noqa: E402

dev = torch.device("cuda", 0)
if len(sys.argv) > 1 and sys.argv[1] == "gpt2":  # the bench.py step instead (GPT-2-small, 64 x 1024)
    from distributedvolunteercomputing_amd.models.gpt2 import GPT2, GPT2Config

    cfg = GPT2Config.preset("gpt2")
    m = GPT2(cfg).to(dev, torch.bfloat16)
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=4), device=dev)
    tok = torch.randint(0, cfg.vocab_size, (64, 1025), device=dev)
    x, y = tok[:, :-1].contiguous(), tok[:, 1:].contiguous()
else:
    m = resnet50().to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    enable_conv_find()
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=4, lr=1e-3, weight_decay=0.0), device=dev)
    tr.compressor = TopKCompressor(tr.flat.numel, 0.01, dev)
    B = 128
    x = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev)
for _ in range(3):
    tr.step(x, y)
torch.cuda.synchronize()
WATCH = ("copy_", "contiguous", "clone", "add", "mul", "sub", "fill_", "zero", "to", "cat", "div", "empty", "full")
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    tr.step(x, y)
    torch.cuda.synchronize()
rows = collections.defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    name = ev.name
    if not name.startswith("aten::") or not any(w in name for w in WATCH):
        continue
    dt = getattr(ev, "device_time_total", None)
    if dt is None:
        dt = getattr(ev, "cuda_time_total", 0.0)
    if dt <= 0:
        continue
    frame = ""
    for f in ev.stack or []:
        if "distributedvolunteercomputing_amd" in f or "cfg3_copy_sources" in f:
            frame = f.split("distributedvolunteercomputing_amd/")[-1]
            break
    key = (name, str(ev.input_shapes)[:110], frame[:90])
    rows[key][0] += 1
    rows[key][1] += dt
for (name, shapes, frame), (n, t) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{t:9.1f} us {n:3d}x  {name:22s} {shapes:110s} {frame}", flush=True)
