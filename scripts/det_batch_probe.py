"""MobileNet-SSD detect() time per 100 frames when the engine runs 1, 2 or 3 chunks (100, 200, 300 frames of
225x400) as ONE batch: the per-layer kernels' last tile wave and the latency-bound extras tail are paid once per
launch, so a worker holding two chunks could run them together. Eager launches, median of interleaved rounds.

    python scripts/det_batch_probe.py [iters]
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.models.mobilenet_ssd import SSDExecutor  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
ex = SSDExecutor(device=dev)
ex.use_graph = False
torch.manual_seed(0)
chunks = {n: torch.randint(0, 256, (n, 225, 400, 3), dtype=torch.uint8, device=dev) for n in (100, 200, 300)}
res = {n: [] for n in chunks}
for n, f in chunks.items():
    ex.detect(f)
torch.cuda.synchronize()
for _ in range(5):
    for n, f in chunks.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            ex.detect(f)
        e1.record()
        torch.cuda.synchronize()
        res[n].append(e0.elapsed_time(e1) / it)
for n, v in res.items():
    med = statistics.median(v)
    print(json.dumps({"frames": n, "detect_ms": round(med, 3), "ms_per_100_frames": round(med * 100 / n, 3)}),
          flush=True)
