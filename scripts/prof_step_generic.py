"""Per-step kernel table of a rocprofv3 --kernel-trace CSV of any trainer step (the last full step,
delimited by the fused AdamW kernel), grouped by kernel name. Usage:
    python scripts/prof_step_generic.py <kernel_trace.csv> [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
idx = [i for i, r in enumerate(rows) if "adamw_flat" in r["Kernel_Name"]]
a, b = (idx[-2] + 1, idx[-1] + 1) if len(idx) >= 2 else (0, len(rows))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[r["Kernel_Name"][:90]][0] += 1
    agg[r["Kernel_Name"][:90]][1] += d
tot = sum(v[1] for v in agg.values())
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"one step: {tot / 1e3:.2f} ms kernel time ({b - a} kernels), first->last kernel span {span / 1e3:.2f} ms")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{v[1] / 1e3:8.3f} ms {v[1] / tot * 100:5.1f}% {v[0]:4d}x  {k}")
