"""Per-kernel summary of the counter passes written by scripts/pmc_step.sh / pmc_gemm.sh.

Columns (per dispatch, medians over dispatches of one kernel name):
  us        duration from the pass's own kernel trace (pass p1)
  rd MB     2 x FETCH_SIZE: on gfx950 FETCH_SIZE counts 64 B per 128-B request of a wide streaming read,
            i.e. half the bytes (MI355X_MICROARCH.md, HBM); includes Infinity-Cache hits
  wr MB     WRITE_SIZE (exact for 16-B-per-lane stores)
  TB/s      (rd + wr) / us
  GHz       effective clock = GRBM_GUI_ACTIVE / 8 XCDs / duration (DVFS under load)
  MFMA %    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): share of all SIMD-cycles the
            matrix pipes were busy (unit: % of the chip's MFMA issue capacity at the held clock)
  VALU %    SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: share of wave-cycles spent issuing VALU (both quad-cycles)
  wait %    SQ_WAIT_ANY / SQ_WAVE_CYCLES: share of wave-cycles parked on s_waitcnt / s_barrier
  stall %   SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES: share of wave-cycles with an instruction not issuable
  VALU/MFMA SQ_INSTS_VALU / SQ_INSTS_MFMA
  LDS cf/in SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS: extra LDS cycles per LDS instruction
A column shows '-' when its pass did not run.

    python scripts/pmc_summary.py gpurun_out/pmc_step > profiles/r6_gpt2_step_pmc.txt
"""
import collections
import csv
import glob
import os
import sys

NSIMD = 1024  # 256 CUs x 4 SIMDs
NXCD = 8


def short(n):
    return n.split("(")[0][:64]


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [v]
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # pass -> kernel -> [GRBM]
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        pas = os.path.relpath(f, d).split(os.sep)[0]
        for r in csv.DictReader(open(f)):
            k, c, v = short(r["Kernel_Name"]), r["Counter_Name"], float(r["Counter_Value"])
            if c == "GRBM_GUI_ACTIVE":
                per[pas][k].append(v)
            else:
                vals[k][c].append(v)
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "p1", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return vals, per, durs


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def fmt(x, spec):
    return format(x, spec) if x == x else "-".rjust(int(spec.split(".")[0]) if spec[0].isdigit() else 1)


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_step"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    vals, per, durs = load(d)
    rows = []
    for k, c in vals.items():
        n = len(durs.get(k, []))
        t = med(durs.get(k, []))
        g = lambda name: med(c.get(name, []))  # noqa: E731
        rd, wr = 2 * g("FETCH_SIZE") * 1024, g("WRITE_SIZE") * 1024
        grbm1 = med(per.get("p1", {}).get(k, []))
        grbm3 = med(per.get("p3", {}).get(k, []))
        ghz = grbm1 / NXCD / (t * 1e3) if t == t and t > 0 else float("nan")
        mf = g("SQ_VALU_MFMA_BUSY_CYCLES")
        mfu = 100 * mf / (NSIMD * grbm3 / NXCD) if grbm3 == grbm3 and grbm3 > 0 else float("nan")
        wc = g("SQ_WAVE_CYCLES")
        valu = 100 * g("SQ_ACTIVE_INST_VALU") / wc if wc == wc and wc > 0 else float("nan")
        wait = 100 * g("SQ_WAIT_ANY") / wc if wc == wc and wc > 0 else float("nan")
        stall = 100 * g("SQ_WAIT_INST_ANY") / wc if wc == wc and wc > 0 else float("nan")
        nm = g("SQ_INSTS_MFMA")
        vpm = g("SQ_INSTS_VALU") / nm if nm == nm and nm > 0 else float("nan")
        lds = g("SQ_INSTS_LDS")
        bc = g("SQ_LDS_BANK_CONFLICT") / lds if lds == lds and lds > 0 else float("nan")
        bw = (rd if rd == rd else 0) + (wr if wr == wr else 0)
        bw = bw / (t * 1e-6) / 1e12 if t == t and t > 0 and (rd == rd or wr == wr) else float("nan")
        rows.append((n * t if t == t else 0, k, n, t, rd, wr, bw, ghz, mfu, valu, wait, stall, vpm, bc))
    rows.sort(reverse=True)
    hdr = (f"{'kernel':64s} {'n':>4s} {'us':>8s} {'rd MB':>8s} {'wr MB':>8s} {'TB/s':>5s} {'GHz':>5s} {'MFMA%':>6s} "
           f"{'VALU%':>6s} {'wait%':>6s} {'stall%':>6s} {'V/MFMA':>7s} {'LDScf':>6s}")
    print(hdr)
    for r in rows[:top]:
        _, k, n, t, rd, wr, bw, ghz, mfu, valu, wait, stall, vpm, bc = r
        print(f"{k:64s} {n:4d} {fmt(t, '8.1f')} {fmt(rd / 1e6, '8.1f')} {fmt(wr / 1e6, '8.1f')} {fmt(bw, '5.2f')} "
              f"{fmt(ghz, '5.2f')} {fmt(mfu, '6.1f')} {fmt(valu, '6.1f')} {fmt(wait, '6.1f')} {fmt(stall, '6.1f')} "
              f"{fmt(vpm, '7.2f')} {fmt(bc, '6.3f')}")


if __name__ == "__main__":
    main()
