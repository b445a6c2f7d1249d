"""Kernel statistics from a rocprofv3 SQLite database (rocprofv3 --kernel-trace without
--output-format csv writes only <name>_results.db): name | calls | avg us | min | max | share,
the same columns as the csv-derived profiles/*_kernel_stats.txt (developer tool).
A third argument "gaps" adds the idle time between consecutive dispatches on one queue
(start of a kernel minus the end of the one before it), per kernel name and overall."""
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

if len(sys.argv) > 3 and sys.argv[3] == "gaps":
    cols = [r[1] for r in db.execute("pragma table_info(kernels)").fetchall()]
    q = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    sel = f"select name, start, end{', ' + q if q else ''} from kernels order by start"
    prev = {}
    gaps = {}
    for row in db.execute(sel):
        name, st, en = row[0], row[1], row[2]
        key = row[3] if q else 0
        if key in prev:
            g = st - prev[key]
            if 0 <= g < 100000:  # same burst (< 100 us): a launch boundary, not host idle
                gaps.setdefault(name, []).append(g)
        prev[key] = en
    allg = [g for v in gaps.values() for g in v]
    print(f"# gaps before a dispatch on the same {q or 'device'} (< 100 us): n {len(allg)}, "
          f"avg {sum(allg) / max(1, len(allg)) / 1e3:.2f} us")
    print("# name | gaps | avg gap us | min | max")
    for name, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:n]:
        print(f"{name} | {len(v)} | {sum(v) / len(v) / 1e3:.2f} | {min(v) / 1e3:.2f} | {max(v) / 1e3:.2f}")
