"""One volunteer's 100-frame chunk on the GPU, stage by stage (HIP-event spans) and as a kernel
trace when run under rocprofv3: 720p synthetic frames -> engine (H2D, resize, detect, annotate,
D2H), then the network alone on pre-resized frames.

    python scripts/video_chunk_prof.py [iters]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.io.video import synthetic_frame  # noqa: E402
from distributedvolunteercomputing_amd.jobs.video import DetectorEngine  # noqa: E402
from distributedvolunteercomputing_amd.ops import vision as V  # noqa: E402
from distributedvolunteercomputing_amd.utils.trace import SpanTracer  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
eng = DetectorEngine(device=dev)
frames = np.stack([synthetic_frame(i, 1280, 720) for i in range(100)])
for _ in range(2):
    eng.process(frames, "127.0.0.1:5554")
torch.cuda.synchronize()
eng.tracer = SpanTracer("engine", enabled=True)
t0 = time.perf_counter()
for _ in range(it):
    eng.process(frames, "127.0.0.1:5554")
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / it * 1e3
eng.tracer.flush()
spans = {k: round(v[1] / v[0], 3) for k, v in eng.tracer.totals.items()}
small = V.resize_width(torch.from_numpy(frames).to(dev), 400).contiguous()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    eng.exec.detect(small)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"engine_wall_ms_per_chunk": round(wall, 2), "span_ms": spans,
                  "net_only_ms": round(e0.elapsed_time(e1) / it, 3)}), flush=True)
