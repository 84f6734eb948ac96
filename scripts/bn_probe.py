"""Train-mode BatchNorm kernels (csrc/kernels/batchnorm.hip) at every distinct ResNet-50 BN shape of config 3 (B=128,
channels-last bf16), forward (stats + apply with the ReLU mask) and backward (reduce + dx), each shape called 20 times
with its own layer workspace -- run under `rocprofv3 --kernel-trace` to get per-dispatch durations by shape
(scripts/bn_probe_summary.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C_ = native()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
SHAPES = [(112, 64), (56, 64), (56, 256), (56, 128), (28, 128), (28, 512), (28, 256), (14, 256), (14, 1024),
          (14, 512), (7, 512), (7, 2048)]
for hw, c in SHAPES:
    x = torch.randn(B, hw, hw, c, device="cuda", dtype=torch.bfloat16)
    g = torch.ones(c, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(c, device="cuda", dtype=torch.bfloat16)
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    lws = torch.zeros(4 * c, device="cuda")
    dy = torch.randn_like(x)
    for _ in range(20):
        lws[: 2 * c].zero_()
        y, mean, rstd, scale, mask = C_.bn_fwd_train(x, None, g, b, rm, rv, 1e-5, 0.1, True, None, lws)
        lws[2 * c:].zero_()
        C_.bn_bwd(dy, mask, x, mean, rstd, scale, True, False, None, None, lws)
    torch.cuda.synchronize()
    print(f"shape {hw}^2 x {c}: {B * hw * hw * c * 2 / 1e6:.1f} MB", flush=True)
