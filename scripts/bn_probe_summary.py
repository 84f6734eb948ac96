"""Median duration per (shape, kernel) of a rocprofv3 kernel-trace CSV of scripts/bn_probe.py (shapes in launch order,
20 iterations each) with the implied TB/s of the bytes each kernel must move: stats reads x; apply reads x, writes y
and the 1-bit mask; bwd_reduce reads dy, x, mask; bwd_dx reads dy, x, mask and writes dx."""
import collections
import csv
import statistics
import sys

SHAPES = [(112, 64), (56, 64), (56, 256), (56, 128), (28, 128), (28, 512), (28, 256), (14, 256), (14, 1024),
          (14, 512), (7, 512), (7, 2048)]
B = 128
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
KS = ("stats_kernel", "apply_kernel", "bwd_reduce_kernel", "bwd_dx_kernel")
res = collections.OrderedDict()
nstats = 0
for r in rows:
    n = r["Kernel_Name"]
    k = next((k for k in KS if k in n), None)
    if k is None:
        continue
    if k == "stats_kernel":
        nstats += 1
    si = (nstats - 1) // 20
    res.setdefault((si, k), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
tot = collections.Counter()
for (si, k), ts in res.items():
    hw, c = SHAPES[si]
    mb = B * hw * hw * c * 2 / 1e6
    moved = {"stats_kernel": 1, "apply_kernel": 2 + 1 / 16, "bwd_reduce_kernel": 2 + 1 / 16,
             "bwd_dx_kernel": 3 + 1 / 16}[k] * mb
    t = statistics.median(ts)
    tot[k] += t
    print(f"{hw:3d}^2 x {c:4d} ({mb:6.1f} MB)  {k:18s} {t:7.1f} us  {moved / t:5.2f} TB/s")
print("sum of medians per kernel (one call per shape):", {k: round(v, 1) for k, v in tot.items()})
