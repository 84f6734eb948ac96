"""The MobileNet-SSD pointwise layers (100-frame chunk) on every GEMM path we have: gemm_nt with the
bias+ReLU epilogue (the executor's default where it tiles), the vision gemm_bias_act (128 x 128
tiles), the library GEMM + a ReLU pass, and gemm_ps on a 256-row-padded activation (bias epilogue
only; an estimate of the persistent kernel at these shapes). Median microseconds per call.

    python scripts/detector_pw_shapes.py
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_ps_bench import timeit  # noqa: E402
from distributedvolunteercomputing_amd.ops import native  # noqa: E402

C = native()
dev = "cuda"
bf = torch.bfloat16
F_ = 100  # frames per chunk
SHAPES = [("conv2 75x75", 75 * 75, 128, 64), ("conv3 75x75", 75 * 75, 128, 128),
          ("conv4 38x38", 38 * 38, 256, 128), ("conv5 38x38", 38 * 38, 256, 256),
          ("conv6 19x19", 19 * 19, 512, 256), ("conv7 19x19", 19 * 19, 512, 512),
          ("conv12 10x10", 10 * 10, 1024, 512), ("conv13 10x10", 10 * 10, 1024, 1024)]


def main():
    torch.manual_seed(0)
    for name, hw, n, k in SHAPES:
        m = F_ * hw
        mp = (m + 255) // 256 * 256
        xa = torch.randn(mp, k, device=dev, dtype=bf)
        x = xa[:m]
        w = torch.randn(n, k, device=dev, dtype=bf) * 0.05
        b32 = torch.randn(n, device=dev, dtype=torch.float32) * 0.1
        b16 = b32.to(bf)
        y = torch.empty(m, n, device=dev, dtype=bf)
        yp = torch.empty(mp, n, device=dev, dtype=bf)
        fns, names = [], []
        if C.gemm_nt_supported_epi(m, n, k, 4):
            fns.append(lambda: C.gemm_nt(x, w, y, None, b16, None, 4))
            names.append("gemm_nt")
        fns.append(lambda: C.gemm_bias_act(x, w, b32, True))
        names.append("gemm_bias_act")
        fns.append(lambda: F.relu_(F.linear(x, w, b16)))
        names.append("library+relu")
        if C.gemm_ps_supported(mp, n, k, 1):
            fns.append(lambda: C.gemm_ps(xa, w, yp, None, b16, None, 1))
            names.append("gemm_ps(pad)")
        ts = timeit(fns, rounds=7, it=20)
        fl = 2.0 * m * n * k
        mb = (m * k + m * n + n * k) * 2 / 1e6
        print(f"{name:13s} M={m:6d} N={n:5d} K={k:5d} ({mb:5.0f} MB) " +
              "  ".join(f"{nm} {t:6.1f} us ({fl / t / 1e6:4.0f} TF)" for nm, t in zip(names, ts)), flush=True)


if __name__ == "__main__":
    main()
