"""Kernel table from a rocprofv3 results database (rocpd sqlite): per-kernel statistics, or with
--sequence START_KERNEL the dispatch sequence of the last pass that begins with that kernel.

    python scripts/rocpd_kernels.py gpurun_out/x/prof/run_results.db [--sequence blob_bilinear]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--sequence", default=None)
    ap.add_argument("--end", default=None, help="kernel name that ends the sequence (inclusive)")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, start, end, grid_x, grid_y, grid_z from kernels order by start").fetchall()
    short = lambda n: n.split("(")[0][:60]  # noqa: E731
    if a.sequence:
        # the last occurrence that starts a pass (is followed by a different kernel)
        starts = [i for i, r in enumerate(rows) if a.sequence in r[0] and i + 1 < len(rows)
                  and a.sequence not in rows[i + 1][0]]
        i0 = starts[-1]
        seq = []
        for r in rows[i0:]:
            seq.append(r)
            if a.end and a.end in r[0] and len(seq) > 1:
                break
        t0 = seq[0][1]
        tot = 0.0
        for n, s, e, gx, gy, gz in seq:
            us = (e - s) / 1e3
            tot += us
            print(f"{(s - t0) / 1e3:9.1f} {us:8.1f} us  grid {gx}x{gy}x{gz}  {short(n)}")
        print(f"sum of kernel times {tot:.1f} us, span {(seq[-1][2] - t0) / 1e3:.1f} us")
        return
    st = collections.defaultdict(list)
    for n, s, e, *_ in rows:
        st[short(n)].append((e - s) / 1e3)
    for n, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):6d} {sum(v):10.1f} us  mean {sum(v) / len(v):8.1f}  {n}")


if __name__ == "__main__":
    main()
