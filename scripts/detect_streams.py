"""Device time of the MobileNet-SSD network per 100 frames when the chunk runs as one pass or as S
slices of 100/S frames on S concurrent streams (each layer's small GEMMs and depthwise passes leave
part of the chip idle in their tails; concurrent slices fill those gaps).

    python scripts/detect_streams.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.io.video import synthetic_frame  # noqa: E402
from distributedvolunteercomputing_amd.jobs.video import DetectorEngine  # noqa: E402
from distributedvolunteercomputing_amd.ops import vision as V  # noqa: E402

dev = torch.device("cuda", 0)
eng = DetectorEngine(device=dev)
frames = np.stack([synthetic_frame(i, 1280, 720) for i in range(100)])
small = V.resize_width(torch.from_numpy(frames).to(dev), 400).contiguous()
ex = eng.exec
ref_dets, ref_cnt = ex.detect(small)
torch.cuda.synchronize()
res = {}
for S in (1, 2, 4):
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    parts = small.chunk(S)

    def run():
        main = torch.cuda.current_stream(dev)
        outs = []
        for st, p in zip(streams, parts):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                outs.append(ex.detect(p))
        for st in streams:
            main.wait_stream(st)
        return outs

    for _ in range(3):
        outs = run()
    torch.cuda.synchronize()
    cnt = torch.cat([o[1] for o in outs])
    res[f"streams_{S}_count_diffs"] = int((cnt.cpu() != ref_cnt.cpu()).sum())  # split-K order may differ
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    res[f"streams_{S}_ms"] = round(sorted(ts)[3], 3)
    print(json.dumps(res), flush=True)
