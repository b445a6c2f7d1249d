"""Summarise a rocprofv3 kernel_stats.csv: per-kernel totals and per-decode-step share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    t = float(r["TotalDurationNs"])
    per = f" {t / steps / 1e3:8.1f}us/step" if steps else ""
    print(f"{t / 1e6:9.2f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:>6} avg={float(r['AverageNs']) / 1e3:9.2f}us{per}  {r['Name'][:90]}")
print(f"total {tot / 1e6:.2f} ms")
