"""Per-step kernel-time table by CATEGORY from a rocprofv3 --kernel-trace CSV (the last full step,
delimited by the fused AdamW kernel), plus the top kernels by full name.
Usage: python scripts/prof_categories.py <kernel_trace.csv> [top-N]"""
import collections
import csv
import re
import sys

CATS = [  # first match wins
    ("implicit-GEMM conv / forward GEMM (HIP gemm_f)", r"gemm_f::|gemm_f_kernel"),
    ("BN (HIP batchnorm.hip)", r"vcx::bn::|stats_kernel|finalize_kernel|apply_kernel|bwd_reduce_kernel|bwd_dx_kernel"),
    ("max-pool (HIP)", r"maxpool"),
    ("weight-gradient GEMM (HIP gemm_wg)", r"gemm_wg"),
    ("persistent GEMM (HIP gemm_ps)", r"gemm_ps"),
    ("conv wgrad (MIOpen)", r"(?i)wrw|bwd_weight|BackwardWeights|conv.*wei"),
    ("conv dgrad (MIOpen)", r"(?i)bwd_data|BackwardData|conv.*bwd|igemm_bwd|dgrad"),
    ("conv fwd (MIOpen)", r"(?i)conv|igemm_fwd|MIOpen|naive"),
    ("library GEMM (1x1 conv / fc)", r"Cijk|gemm|GEMM"),
    ("top-k / compression (HIP)", r"topk|hist|radix|select|psgd_"),
    ("AdamW / local-SGD (HIP)", r"adamw|adam_prologue|grad_sumsq|lsgd"),
    ("split-K / colsum / transpose (HIP)", r"splitk|colsum|transpose|add_f32"),
    ("attention (HIP)", r"attn_"),
    ("LayerNorm / xent (HIP)", r"ln_fwd|ln_bwd|xent"),
    ("torch elementwise / reductions", r"elementwise|reduce_kernel|Fill|copy|Reduce|vectorized"),
]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    idx = [i for i, r in enumerate(rows) if "adamw_flat" in r["Kernel_Name"]]
    a, b = (idx[-2] + 1, idx[-1] + 1) if len(idx) >= 2 else (0, len(rows))
    cat = collections.defaultdict(lambda: [0, 0.0])
    name = collections.defaultdict(lambda: [0, 0.0])
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        n = r["Kernel_Name"]
        c = next((c for c, rx in CATS if re.search(rx, n)), "other")
        cat[c][0] += 1
        cat[c][1] += d
        name[n][0] += 1
        name[n][1] += d
    tot = sum(v[1] for v in cat.values())
    print(f"one step: {tot / 1e3:.2f} ms kernel time ({b - a} kernels)")
    for c, v in sorted(cat.items(), key=lambda x: -x[1][1]):
        print(f"{v[1] / 1e3:8.3f} ms {v[1] / tot * 100:5.1f}% {v[0]:4d}x  {c}")
    print(f"\ntop {top} kernels:")
    for n, v in sorted(name.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{v[1] / 1e3:8.3f} ms {v[0]:4d}x  {n[:110]}")


if __name__ == "__main__":
    main()
