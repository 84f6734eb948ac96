"""Per-step kernel-time summary of a rocprofv3 --kernel-trace of bench.py (last full step,
delimited by the fused AdamW kernel). Usage: python scripts/prof_summary.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if "adamw_flat" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
# first match wins: specific names before the generic ones they contain ("splitk_reduce_kernel" is ours,
# "reduce_kernel" alone is torch's)
KEYS = ["attn_hm_fwd", "attn_hm_dq", "attn_hm_dkv", "attn_fwd", "attn_bwd_dq", "attn_bwd_dkdv", "attn_bwd_delta",
        "ln_fwd", "ln_bwd", "bias_gelu_fwd", "bias_gelu_bwd", "xent_fwd", "xent_bwd", "embed_fwd", "embed_bwd",
        "colsum", "adamw", "grad_sumsq", "splitk_reduce", "psgd_", "swiglu", "rope_qkv", "FillFunctor",
        "distribution_elementwise", "reduce_kernel", "elementwise", "copyBuffer", "fillBuffer", "adam_prologue",
        "xent_fused", "gemm_ps_kernel", "gemm_nt_kernel", "transpose_bf16", "bn_", "stats_kernel", "apply_kernel"]


def short(n):
    for k in KEYS:
        if k in n:
            return k
    return "GEMM " + n[:48]


agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = short(r["Kernel_Name"])
    agg[k][0] += 1
    agg[k][1] += d
tot = sum(v[1] for v in agg.values())
gemm = sum(v[1] for k, v in agg.items() if k.startswith("GEMM"))
print(f"one step: {tot / 1e3:.2f} ms kernel time ({b - a} kernels), GEMM {gemm / 1e3:.2f} ms")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{v[1] / 1e3:8.3f} ms {v[1] / tot * 100:5.1f}% {v[0]:4d}x  {k}")
