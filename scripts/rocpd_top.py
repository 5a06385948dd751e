"""Per-kernel summary (calls, average and total device time) from a rocprofv3 SQLite output
(run_results.db; the default output format of ROCm 7's rocprofv3).  usage: rocpd_top.py DB [N] [DIVISOR]
DIVISOR: divide the call counts and totals by it (e.g. the number of identical calls profiled)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
div = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = db.execute(f"select {name}, count(*), avg(end - start), sum(end - start) from kernels group by {name} "
                  "order by sum(end - start) desc").fetchall()
tot = sum(r[3] for r in rows)
for k, c, a, s in rows[:n]:
    print(f"{k[:88]:88s} calls={c / div:8.1f} avg_us={a / 1e3:8.2f} tot_ms={s / 1e6 / div:8.3f} pct={100 * s / tot:5.1f}")
print(f"total device ms {tot / 1e6 / div:.3f}")
