"""print the top kernels of a rocprofv3 kernel_stats.csv (developer tool)"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 22
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    print(f"{r['Name'][:80]:80s} calls {r['Calls']:>6s} avg {float(r['AverageNs'])/1000:8.2f} us "
          f"tot {float(r['TotalDurationNs'])/1e6:8.2f} ms")
