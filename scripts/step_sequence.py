"""The kernels of the last full step of a rocprofv3 kernel-trace CSV in launch order (one line each: start offset,
duration, grid, name), delimited by the fused AdamW kernel, with the neighbours of every kernel whose name matches
the pattern marked -- to see where copies and fills come from.  python scripts/step_sequence.py trace.csv [regex]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"copyBuffer|Fill|fillBuffer|elementwise")
idx = [i for i, r in enumerate(rows) if "adamw_flat" in r["Kernel_Name"]]
lo, hi = (idx[-2] + 1, idx[-1] + 1) if len(idx) >= 2 else (0, len(rows))
t0 = int(rows[lo]["Start_Timestamp"])
for i in range(lo, hi):
    r = rows[i]
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    mark = ">>" if pat.search(r["Kernel_Name"]) else "  "
    print(f"{mark} {(int(r['Start_Timestamp']) - t0) / 1000:9.1f} {us:8.1f} {r.get('Grid_Size', r.get('Grid_Size_X', '')):>9} "
          f"{r['Kernel_Name'][:110]}")
