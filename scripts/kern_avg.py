"""Mean duration (us) of the last N dispatches of kernels matching a
pattern in rocprofv3 sqlite outputs: scripts/kern_avg.py DB PATTERN [N]."""
import sqlite3
import sys

db, pat = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
c = sqlite3.connect(db)
names = sorted({r[0] for r in c.execute("select name from kernels where name like ?",
                                          (f"%{pat}%",))})
for name in names:
    d = [r[0] / 1000.0 for r in c.execute(
        "select end - start from kernels where name = ? order by start", (name,))][-n:]
    print(f"{name[:60]:60s} last{len(d)} mean {sum(d) / max(len(d), 1):9.1f} us")
