"""Same-process A/B of the MobileNet-SSD network on one 100-frame chunk: the one-launch SSD tail
(VCX_SSD_TAIL=1, csrc/kernels/ssd_tail.hip) vs the per-layer extras + side-stream heads (=0).
Interleaved rounds, median wall time of the forward pass (device-synchronised)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.models.mobilenet_ssd import SSDExecutor  # noqa: E402
from distributedvolunteercomputing_amd.ops import vision as V  # noqa: E402

dev = torch.device("cuda", 0)
exs = {}
for v in ("0", "1", "chain"):
    os.environ["VCX_SSD_TAIL"] = v
    exs[v] = SSDExecutor(device=dev)
torch.manual_seed(0)
frames = torch.randint(0, 256, (100, 225, 400, 3), dtype=torch.uint8, device=dev)
blob = V.blob_from_frames(frames, 300)
res = {v: [] for v in exs}
for v, ex in exs.items():
    for _ in range(3):
        ex.forward_blob(blob)
torch.cuda.synchronize()
for rnd in range(7):
    for v, ex in exs.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            ex.forward_blob(blob)
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / 10 * 1e3)
for v, ts in res.items():
    print(f"VCX_SSD_TAIL={v}: network {sorted(ts)[len(ts) // 2]:.3f} ms per 100-frame chunk (rounds "
          f"{', '.join('%.3f' % t for t in ts)})", flush=True)
# per-step split with events (the tail as one step)
for v in ("1", "chain"):
    steps = exs[v].step_times(blob, 10)
    tail = [s for s in steps if s[1] == "tail"]
    print(f"VCX_SSD_TAIL={v} tail step:", tail, " sum of steps %.3f ms" % sum(s[2] for s in steps), flush=True)
