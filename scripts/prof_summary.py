"""Summarise rocprofv3 output (kernel-trace stats or PMC counters) into a
small markdown table for ``profiles/``.

usage: python scripts/prof_summary.py <rocprof output dir> [--filter SUBSTR] [--top N]

Reads the SQLite database (``*_results.db``) or the CSV files rocprofv3
writes; kernel names are shortened to their leading identifier.
"""
import argparse
import collections
import csv
import glob
import os
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:90]


def load(d):
    counters = collections.defaultdict(lambda: collections.defaultdict(float))
    kernels = collections.defaultdict(list)
    for db in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        con = sqlite3.connect(db)
        cur = con.cursor()
        try:
            for name, cname, val in cur.execute(
                    "select kernel_name, counter_name, value from counters_collection"):
                counters[short(name)][cname] += float(val)
        except sqlite3.OperationalError:
            pass
        try:
            for name, dur in cur.execute("select name, duration from kernels"):
                kernels[short(name)].append(float(dur))
        except sqlite3.OperationalError:
            pass
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            counters[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kernels[short(r["Kernel_Name"])].append(
                float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return counters, kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--filter", default="")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    counters, kernels = load(a.dir)
    if kernels:
        tot = sum(sum(v) for v in kernels.values())
        print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
        for k, v in sorted(kernels.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
            if a.filter in k:
                print(f"| `{k}` | {len(v)} | {sum(v) / 1e6:.3f} | {sum(v) / len(v) / 1e3:.1f} | "
                      f"{100 * sum(v) / tot:.1f} |")
    if counters:
        print("\n| kernel | counter | value |\n|---|---|---|")
        for k, cs in counters.items():
            if a.filter not in k:
                continue
            for c, v in sorted(cs.items()):
                print(f"| `{k}` | {c} | {v:.4g} |")
            if cs.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in cs:
                print(f"| `{k}` | VALU/MFMA (incl. MFMA) | {cs['SQ_INSTS_VALU'] / cs['SQ_INSTS_MFMA']:.2f} |")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "GRBM_GUI_ACTIVE" in cs:
                # busy cycles are summed over all SIMDs (1024) ; GRBM over 8 XCDs
                simd_cyc = cs["GRBM_GUI_ACTIVE"] / 8 * 1024
                print(f"| `{k}` | MFMA busy (of SIMD-cycles) | "
                      f"{100 * cs['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cyc:.1f}% |")


if __name__ == "__main__":
    main()
