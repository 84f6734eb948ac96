"""Per-kernel summary of the counter passes written by scripts/pmc_step.sh.

For each kernel (name up to its argument list): dispatches, median duration (from the pass's own
kernel trace), HBM bytes read / written per dispatch (FETCH_SIZE / WRITE_SIZE are in KiB),
the achieved HBM rate, and MFMA busy / LDS bank-conflict ratios where that pass ran.

    python scripts/pmc_summary.py gpurun_out/pmc_step > profiles/r1_gpt2_step_pmc.txt
"""
import collections
import csv
import glob
import os
import sys


def short(n):
    n = n.split("(")[0]
    return n[:70]


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [v]
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "p1", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return vals, durs


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_step"
    vals, durs = load(d)
    rows = []
    for k, c in vals.items():
        n = len(durs.get(k, []))
        t = med(durs.get(k, []))
        rd = med(c.get("FETCH_SIZE", [])) * 1024
        wr = med(c.get("WRITE_SIZE", [])) * 1024
        busy = med(c.get("SQ_BUSY_CYCLES", []))
        mf = med(c.get("SQ_VALU_MFMA_BUSY_CYCLES", []))
        lds = med(c.get("SQ_INSTS_LDS", []))
        bc = med(c.get("SQ_LDS_BANK_CONFLICT", []))
        rows.append((n * t, k, n, t, rd, wr, mf, busy, lds, bc))
    rows.sort(reverse=True)
    print(f"{'kernel':70s} {'n':>4s} {'us':>8s} {'rd MB':>8s} {'wr MB':>8s} {'TB/s':>6s} "
          f"{'MFMA busy':>10s} {'LDS confl/inst':>14s}")
    for _, k, n, t, rd, wr, mf, busy, lds, bc in rows[:40]:
        bw = (rd + wr) / (t * 1e-6) / 1e12 if t == t and t > 0 else float("nan")
        mfr = mf / busy if busy == busy and busy > 0 and mf == mf else float("nan")
        bcr = bc / lds if lds == lds and lds > 0 and bc == bc else float("nan")
        print(f"{k:70s} {n:4d} {t:8.1f} {rd / 1e6:8.1f} {wr / 1e6:8.1f} {bw:6.2f} {mfr:10.3f} {bcr:14.3f}")


if __name__ == "__main__":
    main()
