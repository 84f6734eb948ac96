"""Median duration per kernel name (full, with template args) from a rocprofv3 kernel trace csv."""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if pat in n:
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items(), key=lambda x: -sorted(x[1])[len(x[1]) // 2]):
    v.sort()
    print(f"{v[len(v) // 2]:9.1f} us  n={len(v):3d}  {n[:110]}")
