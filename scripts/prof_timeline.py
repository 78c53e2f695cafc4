"""Per-iteration GPU timeline from a rocprofv3 kernel trace: busy vs idle
time between consecutive launches of a marker kernel (default: the E-step).

usage: python scripts/prof_timeline.py <rocprof dir> [--marker estep_kernel] [--last N]

Prints, for the last N marker-to-marker intervals, wall / kernel-busy / idle
microseconds, then the kernel sequence of the final interval with the idle
gap in front of each launch (host launch latency and sync bubbles show up
as gaps).
"""
import argparse
import csv
import glob
import os
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", name)[:70]


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    if not rows:
        for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
            con = sqlite3.connect(db)
            try:
                for s, e, n in con.execute("select start, end, name from kernels"):
                    rows.append((int(s), int(e), short(n)))
            except sqlite3.OperationalError:
                pass
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="estep_kernel")
    ap.add_argument("--last", type=int, default=5)
    ap.add_argument("--first", type=int, default=None,
                    help="take --last intervals starting at this one (default: the last ones)")
    ap.add_argument("--seq-all", action="store_true",
                    help="print the kernel sequence of every selected interval")
    a = ap.parse_args()
    rows = load(a.dir)
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < 2:
        raise SystemExit("not enough marker kernels")
    print("| interval | wall us | busy us | idle us | launches |\n|---|---|---|---|---|")
    allv = list(zip(marks[:-1], marks[1:]))
    ivs = allv[-a.last:] if a.first is None else allv[a.first:a.first + a.last]
    for n, (i, j) in enumerate(ivs):
        seg = rows[i:j]
        wall = (rows[j][0] - rows[i][0]) / 1e3
        busy = sum(e - s for s, e, _ in seg) / 1e3
        print(f"| {n} | {wall:.1f} | {busy:.1f} | {wall - busy:.1f} | {len(seg)} |")
    for n, (i, j) in enumerate(ivs if a.seq_all else ivs[-1:]):
        print(f"\ninterval {n if a.seq_all else len(ivs) - 1}\n\n| kernel | us | gap before us |\n|---|---|---|")
        prev = rows[i - 1][1] if i > 0 else rows[i][0]
        for s, e, nme in rows[i:j]:
            print(f"| `{nme}` | {(e - s) / 1e3:.1f} | {(s - prev) / 1e3:.1f} |")
            prev = e


if __name__ == "__main__":
    main()
