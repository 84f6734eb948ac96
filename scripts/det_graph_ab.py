"""Same-process A/B of the MobileNet-SSD chunk as eager launches vs one HIP graph per chunk shape
(SSDExecutor.use_graph, VCX_VISION_GRAPH): detect() on a 100-frame 225x400 uint8 chunk (blob + network +
detection), median wall time per chunk over interleaved rounds, detections compared."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.models.mobilenet_ssd import SSDExecutor  # noqa: E402

dev = torch.device("cuda", 0)
exs = {"eager": SSDExecutor(device=dev), "graph": SSDExecutor(device=dev)}
exs["eager"].use_graph = False
exs["graph"].use_graph = True
torch.manual_seed(0)
frames = torch.randint(0, 256, (100, 225, 400, 3), dtype=torch.uint8, device=dev)
d0, c0 = exs["eager"].detect(frames)
d1, c1 = exs["graph"].detect(frames)
d1, c1 = exs["graph"].detect(frames)  # replay
torch.cuda.synchronize()
print(f"graph captured: {exs['graph'].use_graph} ({exs['graph'].graph_error}); counts equal: {bool(torch.equal(c0, c1))}; "
      f"dets max diff {float((d0.float() - d1.float()).abs().max()):.3e}", flush=True)
res = {k: [] for k in exs}
for rnd in range(9):
    for k, ex in exs.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            ex.detect(frames)
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 10 * 1e3)
for k, ts in res.items():
    print(f"{k}: {sorted(ts)[len(ts) // 2]:.3f} ms per 100-frame chunk (rounds {', '.join('%.3f' % t for t in ts)})",
          flush=True)
