"""Where the requester's host time goes per 100-frame 720p chunk (frame source, gather into
pinned staging, H2D, resize, readback)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributedvolunteercomputing_amd.io.video import synthetic_frame
from distributedvolunteercomputing_amd.ops import vision as V

dev = torch.device("cuda", 0)
fr = [synthetic_frame(i, 1280, 720) for i in range(100)]
t = time.perf_counter()
fr = [synthetic_frame(i, 1280, 720) for i in range(100)]
print(f"synthetic_frame: {(time.perf_counter() - t) * 10:.3f} ms/frame")
pin = torch.empty((100, 720, 1280, 3), dtype=torch.uint8, pin_memory=True)
for rep in range(3):
    t = time.perf_counter()
    for i, f in enumerate(fr):
        pin[i].copy_(torch.from_numpy(f))
    print(f"gather into pinned (torch copy_): {(time.perf_counter() - t) * 1e3:.1f} ms/chunk")
pn = pin.numpy()
for rep in range(2):
    t = time.perf_counter()
    for i, f in enumerate(fr):
        np.copyto(pn[i], f)
    print(f"gather into pinned (np.copyto): {(time.perf_counter() - t) * 1e3:.1f} ms/chunk")
for rep in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    x = pin.to(dev, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    small = V.resize_width(x, 400)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out = torch.empty(small.shape, dtype=torch.uint8, pin_memory=True)
    out.copy_(small)
    t3 = time.perf_counter()
    print(f"H2D {(t1 - t) * 1e3:.2f} ms, resize {(t2 - t1) * 1e3:.2f} ms, D2H {(t3 - t2) * 1e3:.2f} ms")
