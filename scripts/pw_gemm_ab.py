"""Same-process A/B of the MobileNet-SSD pointwise-GEMM choice (VCX_VISION_PW): gemm_nt 256 x 256 tiles
everywhere it applies (nt), the 128 x 128-tile vision GEMM everywhere (vision), or gemm_nt except where its
last wave of tiles leaves most CUs idle (auto, models/mobilenet_ssd.py _nt_tail_bound). Median network time
per 100-frame chunk over interleaved rounds, outputs compared against the nt executor."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.models.mobilenet_ssd import SSDExecutor  # noqa: E402
from distributedvolunteercomputing_amd.ops import vision as V  # noqa: E402

dev = torch.device("cuda", 0)
exs = {}
for v in ("nt", "vision", "auto"):
    os.environ["VCX_VISION_PW"] = v
    exs[v] = SSDExecutor(device=dev)
torch.manual_seed(0)
frames = torch.randint(0, 256, (100, 225, 400, 3), dtype=torch.uint8, device=dev)
blob = V.blob_from_frames(frames, 300)
ref = exs["nt"].forward_blob(blob)
for v, ex in exs.items():
    out = ex.forward_blob(blob)
    for name in ("conv11", "conv13", "mbox_conf"):
        a, r = out[name].float(), ref[name].float()
        print(f"{v}: {name} rel diff vs nt {float((a - r).norm() / (r.norm() + 1e-6)):.2e}", flush=True)
    d0, c0 = ref["detection_out"]
    d1, c1 = out["detection_out"]
    print(f"{v}: detections per frame equal to nt: {bool(torch.equal(c0, c1))}", flush=True)
res = {v: [] for v in exs}
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
    print(f"VCX_VISION_PW={v}: network {sorted(ts)[len(ts) // 2]:.3f} ms per 100-frame chunk "
          f"(rounds {', '.join('%.3f' % t for t in ts)})", flush=True)
