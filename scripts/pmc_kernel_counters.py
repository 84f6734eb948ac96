"""All counters of one kernel (name substring) from rocprofv3 --pmc passes: mean per dispatch.
Usage: python scripts/pmc_kernel_counters.py <pmc dir> <kernel substring>"""
import collections
import csv
import glob
import sys

d, pat = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
