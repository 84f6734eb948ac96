"""Per-layer GPU time of the MobileNet-SSD plan on one 100-frame chunk (HIP events between plan
steps, mean over passes), with the bytes each step must move at minimum and the implied TB/s.

    python scripts/video_layers.py [iters]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.models.mobilenet_ssd import SSDExecutor  # noqa: E402
from distributedvolunteercomputing_amd.ops import vision as V  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
ex = SSDExecutor(device=dev)
torch.manual_seed(0)
frames = torch.randint(0, 256, (100, 225, 400, 3), dtype=torch.uint8, device=dev)
blob = V.blob_from_frames(frames, 300)
steps = ex.step_times(blob, it)
out = ex.forward_blob(blob)
sizes = {k: v.numel() * v.element_size() for k, v in out.items() if torch.is_tensor(v)}
total = 0.0
rows = []
for (name, kind, ms), (kind2, l, _p) in zip(steps, ex._plan):
    total += ms
    if ms < 0.002:
        continue
    mb_in = sizes.get(l.bottoms[0], 0) / 1e6 if l.bottoms else 0.0
    mb_out = sizes.get(l.tops[0], 0) / 1e6 if l.tops else 0.0
    tbs = (mb_in + mb_out) / 1e6 / (ms / 1e3) if ms > 0 else 0.0
    rows.append(dict(layer=name, kind=kind, us=round(ms * 1e3, 1), mb_in=round(mb_in, 1), mb_out=round(mb_out, 1),
                     tb_s=round(tbs, 2)))
    print(f"{name:24s} {kind:6s} {ms * 1e3:8.1f} us  in {mb_in:7.1f} MB  out {mb_out:7.1f} MB  {tbs:5.2f} TB/s",
          flush=True)
by_kind = {}
for r in rows:
    by_kind[r["kind"]] = round(by_kind.get(r["kind"], 0.0) + r["us"], 1)
print(json.dumps({"total_ms": round(total, 3), "by_kind_us": by_kind}), flush=True)

# the same network as the engine runs it: one HIP graph replay per chunk (blob + plan + detection)
for mode in ("graph", "eager"):
    ex.use_graph = mode == "graph"
    ex.detect(frames)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        ex.detect(frames)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"detect_chunk_ms": round(e0.elapsed_time(e1) / it, 3), "mode": mode, "frames": 100}),
          flush=True)
ex.use_graph = True

# preprocessing of the same chunk from 720p: INTER_AREA to 400 px, then the 300x300 blob
big = torch.randint(0, 256, (100, 720, 1280, 3), dtype=torch.uint8, device=dev)
for name, fn in (("resize_area 720p->400", lambda: V.resize_width(big, 400)),
                 ("blob_bilinear 400->300", lambda: V.blob_from_frames(frames, 300))):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        y = fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / it * 1e3
    src = big if name.startswith("resize") else frames
    mb = (src.numel() + y.numel() * y.element_size()) / 1e6
    print(json.dumps({"kernel": name, "us": round(us, 1), "mb": round(mb, 1), "tb_s": round(mb / us, 2)}),
          flush=True)
