"""Per-tensor relative error (Frobenius) of the HIP MobileNet-SSD executor against the fp32 Caffe
reference on the same blob (tests/test_vision_gpu.py::test_executor_matches_caffe_reference)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd.models.mobilenet_ssd import SSDExecutor  # noqa: E402
from distributedvolunteercomputing_amd.ops import vision as V  # noqa: E402

ex = SSDExecutor(device="cuda")
for seed in (4, 5):
    torch.manual_seed(seed)
    frames = torch.randint(0, 256, (2, 225, 400, 3), dtype=torch.uint8, device="cuda")
    blob = V.blob_from_frames(frames, 300)
    out = ex.forward_blob(blob)
    ref = ex.ref(blob[..., :3].permute(0, 3, 1, 2).float().cpu())
    names = ["conv0", "conv1", "conv3", "conv5", "conv7", "conv9", "conv11", "conv13", "conv14_1", "conv14_2",
             "conv15_2", "conv16_2", "conv17_2"]
    row = []
    for name in names:
        a = out[name].float().cpu().permute(0, 3, 1, 2)
        r = ref[name]
        row.append(f"{name} {float((a - r).norm() / (r.norm() + 1e-6)):.4f}")
    for name in ["mbox_loc", "mbox_conf"]:
        a = out[name].float().cpu()
        r = ref[name]
        row.append(f"{name} {float((a - r).norm() / (r.norm() + 1e-6)):.4f}")
    # the bf16 rounding floor: the reference's own tensors rounded to bf16 once
    fl = [f"{n} {float((ref[n].bfloat16().float() - ref[n]).norm() / ref[n].norm()):.4f}" for n in ("conv13", "mbox_conf")]
    print(f"seed {seed}: " + ", ".join(row) + " | one bf16 rounding: " + ", ".join(fl), flush=True)
