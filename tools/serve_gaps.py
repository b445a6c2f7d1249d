"""What the host does while the device idles in a served C4 run (bench.py --stagger).

Reads a rocprofv3 --kernel-trace --hip-trace run (run_kernel_trace.csv, run_hip_api_trace.csv
in one directory): the device's idle gaps are the stretches where no kernel runs (the union of
every queue's kernels); every HIP API call of the host is laid over them.  Prints, per API
function, the idle time its calls overlap (a gap with no API call in it is host code between
calls: Python, the scheduler's bookkeeping), and the API call that enqueued the first kernel
after each gap (by correlation id).
usage: python3 tools/serve_gaps.py DIR [--skip-s S] [--after-setup]
"""
import collections
import csv
import glob
import os
import sys


def rows(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not f:
        sys.exit(f"no {pat} under {d}")
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main():
    d = sys.argv[1]
    skip = float(sys.argv[sys.argv.index("--skip-s") + 1]) if "--skip-s" in sys.argv else 0.0
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Correlation_Id"]), r["Kernel_Name"])
            for r in rows(d, "*kernel_trace.csv")]
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Correlation_Id"]), r["Function"])
           for r in rows(d, "*hip_api_trace.csv")]
    kern.sort()
    api.sort()
    t0 = kern[0][0] + int(skip * 1e9)
    if "--after-setup" in sys.argv:
        # start after the last allocation / queue creation (the warm-up run's setup)
        t0 = max(t0, max(b for a, b, c, f in api if f.startswith(("hipMalloc", "hipStreamCreate", "hipHostMalloc"))))
    kern = [k for k in kern if k[0] >= t0]
    by_corr = {c: f for a, b, c, f in api}
    # idle gaps between the first and the last kernel
    gaps = []
    end = kern[0][1]
    for a, b, c, n in kern[1:]:
        if a > end:
            gaps.append((end, a, by_corr.get(c, "?"), n))
        end = max(end, b)
    wall = end - kern[0][0]
    idle = sum(b - a for a, b, _, _ in gaps)
    print(f"window {wall / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms ({100 * idle / wall:.1f} %) in {len(gaps)} gaps")
    # API time inside the gaps (one sweep; an API call may span several gaps)
    over = collections.Counter()
    calls = collections.Counter()
    covered = 0
    j = 0
    for g0, g1, _, _ in gaps:
        while j < len(api) and api[j][1] <= g0:
            j += 1
        k = j
        iv = []
        while k < len(api) and api[k][0] < g1:
            a, b, c, f = api[k]
            lo, hi = max(a, g0), min(b, g1)
            if hi > lo:
                over[f] += hi - lo
                calls[f] += 1
                iv.append((lo, hi))
            k += 1
        # union of API time in this gap
        iv.sort()
        cur = None
        for lo, hi in iv:
            if cur is None or lo > cur[1]:
                if cur:
                    covered += cur[1] - cur[0]
                cur = [lo, hi]
            else:
                cur[1] = max(cur[1], hi)
        if cur:
            covered += cur[1] - cur[0]
    print(f"  inside HIP API calls {covered / 1e6:.1f} ms, host code between calls {(idle - covered) / 1e6:.1f} ms")
    for f, t in over.most_common(12):
        print(f"     {t / 1e6:8.2f} ms  {calls[f]:7d} calls  {f}")
    print("  the call that enqueued the first kernel after a gap:")
    first = collections.Counter()
    for g0, g1, f, n in gaps:
        first[(f, n[:40])] += g1 - g0
    for (f, n), t in first.most_common(10):
        print(f"     {t / 1e6:8.2f} ms  {f} -> {n}")


if __name__ == "__main__":
    main()
