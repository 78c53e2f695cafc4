"""Per-step GPU kernel time in the timed window of a bench.py run under
rocprofv3 --kernel-trace: the last STEPS steps, delimited by the certified
E-step launches.  usage: scripts/step_kernels.py DB [STEPS] [TOP]"""
import sqlite3
import sys

db = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
x = [i for i, r in enumerate(rows) if "estep_x64" in r[0]]
# bench.py: warmup + STEPS timed + 3 phase-timed steps after them
lo, hi = x[-(steps + 3)] - 8, x[-3] - 8
tot = {}
for n, s, e in rows[lo:hi]:
    k = n.split("(")[0][:60]
    tot[k] = tot.get(k, 0.0) + (e - s) / 1000.0
busy = sum(tot.values())
span = (rows[hi][1] - rows[lo][1]) / 1000.0
print(f"GPU busy {busy / steps:.1f} us/step, span {span / steps:.1f} us/step "
      f"(idle {100 * (1 - busy / span):.1f}%)")
for k, v in sorted(tot.items(), key=lambda t: -t[1])[:top]:
    print(f"{k:60s} {v / steps:8.1f} us/step {100 * v / busy:5.1f}%")

series = {}
for n, s, e in rows[lo:hi]:
    k = n.split("(")[0][:60]
    series.setdefault(k, []).append(int((e - s) / 1000))
for k, v in sorted(tot.items(), key=lambda t: -t[1])[:6]:
    print(f"{k[:40]:40s} per call: {series[k]}")
