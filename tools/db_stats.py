"""Kernel statistics from a rocprofv3 SQLite database (rocprofv3 --kernel-trace without
--output-format csv writes only <name>_results.db): name | calls | avg us | min | max | share,
the same columns as the csv-derived profiles/*_kernel_stats.txt (developer tool)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = db.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                  "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[5] for r in rows)
print("# name | calls | avg us | min us | max us | share of kernel time")
for name, calls, avg, mn, mx, s in rows[:n]:
    print(f"{name} | {calls} | {avg / 1e3:.2f} | {mn / 1e3:.2f} | {mx / 1e3:.2f} | {100.0 * s / tot:.1f}%")
