#!/usr/bin/env python
"""Summarise rocprofv3 sqlite output (rocpd ``*_results.db``) as markdown.

usage: scripts/pmc_summary.py DB [DB ...] [--match SUBSTR] [--top N]

Per kernel (name truncated): dispatches, mean duration, and for PMC runs the
per-dispatch mean of every counter plus derived metrics:
  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  eff. clock = GRBM_GUI_ACTIVE / 8 / duration
"""
import argparse
import collections
import sqlite3
import re


def short(name, n=70):
    name = name.split("(")[0]
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    for db in a.dbs:
        con = sqlite3.connect(db)
        print(f"### {db}\n")
        rows = con.execute("select name, duration from kernels").fetchall()
        agg = collections.defaultdict(list)
        for name, dur in rows:
            agg[name].append(dur)
        tot = sum(sum(v) for v in agg.values()) or 1
        print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
        for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
            print(f"| `{short(name)}` | {len(v)} | {sum(v) / 1e6:.3f} | {sum(v) / len(v) / 1e3:.1f} |"
                  f" {100 * sum(v) / tot:.1f} |")
        try:
            cc = con.execute("select kernel_name, dispatch_id, counter_name, value, duration from "
                             "counters_collection").fetchall()
        except sqlite3.Error:
            cc = []
        if not cc:
            print()
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        durs = collections.defaultdict(dict)
        for kn, did, cn, val, dur in cc:
            if a.match and not re.search(a.match, kn):
                continue
            per[(kn, did)][cn] += val
            durs[kn][did] = dur
        bykern = collections.defaultdict(lambda: collections.defaultdict(list))
        for (kn, did), cnts in per.items():
            for cn, v in cnts.items():
                bykern[kn][cn].append(v)
        print("\n| kernel | counter | mean per dispatch |\n|---|---|---|")
        for kn, cnts in bykern.items():
            mean = {cn: sum(v) / len(v) for cn, v in cnts.items()}
            for cn in sorted(mean):
                print(f"| `{short(kn, 40)}` | {cn} | {mean[cn]:.4g} |")
            d = sum(durs[kn].values()) / max(len(durs[kn]), 1)
            g = mean.get("GRBM_GUI_ACTIVE")
            if g and "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
                print(f"| `{short(kn, 40)}` | MFMA busy (of SIMD-cycles) | "
                      f"{100 * mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.1f}% |")
            if g and d:
                print(f"| `{short(kn, 40)}` | eff. clock GHz | {g / 8 / d:.2f} |")
            if "SQ_INSTS_VALU" in mean and "SQ_INSTS_MFMA" in mean and mean["SQ_INSTS_MFMA"]:
                print(f"| `{short(kn, 40)}` | VALU/MFMA | "
                      f"{mean['SQ_INSTS_VALU'] / mean['SQ_INSTS_MFMA']:.2f} |")
            if "SQ_WAVE_CYCLES" in mean and "SQ_WAIT_INST_ANY" in mean:
                print(f"| `{short(kn, 40)}` | issue-stall share (WAIT_INST_ANY/WAVE_CYCLES) | "
                      f"{100 * mean['SQ_WAIT_INST_ANY'] / mean['SQ_WAVE_CYCLES']:.1f}% |")
            if "SQ_WAVE_CYCLES" in mean and "SQ_WAIT_ANY" in mean:
                print(f"| `{short(kn, 40)}` | parked share (WAIT_ANY/WAVE_CYCLES) | "
                      f"{100 * mean['SQ_WAIT_ANY'] / mean['SQ_WAVE_CYCLES']:.1f}% |")
        print()


if __name__ == "__main__":
    main()
