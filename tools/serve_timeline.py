"""Decompose a served C4 run (bench.py --stagger) from a rocprofv3 kernel trace.

The batched decode steps and the stacked prefills run on the batch queue (the queue that
carries k_argmax_batch_final); the cross-stream encoder passes (mel, conv stems, the 32
layers, adapters) run on the member streams' queues.  Over the traced window this prints:
  * busy time per class (union of its kernels' intervals) and the overlap of steps with
    encoder kernels; idle = no kernel of any class running;
  * the batched step's GPU span (end of one k_argmax_batch_final to the next, for steps that
    follow each other on the queue) split by whether an encoder kernel ran during it;
  * the kernel time per class by kernel (top entries).
usage: python3 tools/serve_timeline.py run_kernel_trace.csv [--skip-s S]
"""
import collections
import csv
import sys

# kernels only the batched step launches: on the batch queue a stacked prefill runs from a
# k_embed_rows to the next of these
STEP_NAMES = ("k_embed_batch", "k_resid_xw_fplanes", "k_skl", "k_sklx", "k_attn_decode", "k_skf", "k_argmax_rows",
              "k_argmax_batch_final", "k_swiglu_fplanes")


def short(name):
    n = name.replace("void ", "").replace("vox::", "")
    return n.split("(")[0]


def union(iv):
    """total length of the union of [a, b) intervals"""
    tot, cur_a, cur_b = 0, None, None
    for a, b in sorted(iv):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def intersect_len(iv, jv):
    """length of (union iv) intersected with (union jv)"""
    ev = []
    for a, b in iv:
        ev.append((a, 0, 1))
        ev.append((b, 0, -1))
    for a, b in jv:
        ev.append((a, 1, 1))
        ev.append((b, 1, -1))
    ev.sort()
    c = [0, 0]
    last, tot = None, 0
    for t, k, d in ev:
        if last is not None and c[0] > 0 and c[1] > 0:
            tot += t - last
        c[k] += d
        last = t
    return tot


def main():
    path = sys.argv[1]
    skip = float(sys.argv[sys.argv.index("--skip-s") + 1]) if "--skip-s" in sys.argv else 0.0
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), short(r["Kernel_Name"])))
    rows.sort()
    t0 = rows[0][0] + int(skip * 1e9)
    rows = [r for r in rows if r[0] >= t0]
    bq = collections.Counter(q for a, b, q, n in rows if n.startswith("k_argmax_batch_final"))
    if not bq:
        sys.exit("no batched steps in the trace")
    batch_q = bq.most_common(1)[0][0]
    # the traced window: first to last batched step kernel
    first = min(a for a, b, q, n in rows if q == batch_q)
    last = max(b for a, b, q, n in rows if q == batch_q)
    rows = [r for r in rows if r[1] > first and r[0] < last]
    cls = collections.defaultdict(list)
    per = collections.defaultdict(lambda: collections.Counter())
    queues = collections.defaultdict(collections.Counter)
    in_prefill = False
    for a, b, q, n in rows:
        if q == batch_q:
            if n.startswith("k_embed_rows"):
                in_prefill = True
            elif n.startswith(STEP_NAMES):
                in_prefill = False
            c = "prefill" if in_prefill else "step"
        else:
            c = "encoder"
        cls[c].append((a, b))
        per[c][n] += b - a
        queues[c][q] += 1
    wall = last - first
    allv = [iv for v in cls.values() for iv in v]
    busy = union(allv)
    print(f"window {wall / 1e6:.1f} ms (first to last batch-queue kernel), batch queue {batch_q}")
    print(f"  any kernel running  {busy / 1e6:9.1f} ms ({100 * busy / wall:5.1f} %)   idle {100 * (wall - busy) / wall:5.1f} %")
    for c in ("step", "prefill", "encoder"):
        u = union(cls[c])
        s = sum(b - a for a, b in cls[c])
        print(f"  {c:8s} busy {u / 1e6:9.1f} ms ({100 * u / wall:5.1f} %)  kernel-sum {s / 1e6:9.1f} ms  launches {len(cls[c])}")
    ov = intersect_len(cls["step"], cls["encoder"])
    print(f"  steps beside encoder kernels {ov / 1e6:.1f} ms ({100 * ov / max(1, union(cls['step'])):.1f} % of step busy)")
    # step spans: k_argmax_batch_final end -> next k_argmax_batch_final end
    ends = sorted(b for a, b, q, n in rows if q == batch_q and n.startswith("k_argmax_batch_final"))
    enc = sorted(cls["encoder"])
    pre = sorted(cls["prefill"])

    def touches(iv, a, b):
        # any interval of iv overlapping [a, b) (iv sorted by start)
        import bisect
        i = bisect.bisect_left(iv, (b, b))
        for j in range(max(0, i - 64), i):
            if iv[j][1] > a and iv[j][0] < b:
                return True
        return False

    spans = {"alone": [], "beside encoder": [], "with prefill": []}
    for e0, e1 in zip(ends, ends[1:]):
        if touches(pre, e0, e1):
            spans["with prefill"].append(e1 - e0)
        elif touches(enc, e0, e1):
            spans["beside encoder"].append(e1 - e0)
        else:
            spans["alone"].append(e1 - e0)
    for k, v in spans.items():
        if v:
            v.sort()
            print(f"  step span {k:15s} n={len(v):5d}  p50 {v[len(v) // 2] / 1e3:8.1f} us  mean {sum(v) / len(v) / 1e3:8.1f} us"
                  f"  sum {sum(v) / 1e6:8.1f} ms")
    for c in ("step", "prefill", "encoder"):
        print(f"  {c} launches by queue id: {dict(queues[c])}")
    if "--dump" in sys.argv:
        # every kernel of the first few step spans that had encoder kernels in them
        shown = 0
        for e0, e1 in zip(ends, ends[1:]):
            if not touches(enc, e0, e1) or touches(pre, e0, e1):
                continue
            print(f"  -- step span {(e1 - e0) / 1e3:.1f} us with encoder kernels (t = 0 at the previous step's end)")
            for a, b, q, n in rows:
                if b > e0 and a < e1:
                    print(f"     q{q:<3d} {(a - e0) / 1e3:9.1f} .. {(b - e0) / 1e3:9.1f} us  {n[:60]}")
            shown += 1
            if shown >= 2:
                break
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 8
    for c in ("step", "prefill", "encoder"):
        tot = sum(per[c].values())
        print(f"  {c}: top kernels")
        for n, t in per[c].most_common(top):
            print(f"     {t / 1e6:8.2f} ms {100 * t / max(1, tot):5.1f} %  {n}")
    # idle gaps: the device runs nothing between the last kernel to end and the next to start;
    # each gap is attributed to (class of the kernel that ended last -> class of the next one)
    # and to the next kernel's name (what the host submitted after the gap)
    labelled = []
    in_prefill = False
    for a, b, q, n in rows:
        if q == batch_q:
            if n.startswith("k_embed_rows"):
                in_prefill = True
            elif n.startswith(STEP_NAMES):
                in_prefill = False
            c = "prefill" if in_prefill else "step"
        else:
            c = "encoder"
        labelled.append((a, b, c, n))
    gaps = collections.Counter()
    gapn = collections.Counter()
    sizes = collections.Counter()
    end, endc = labelled[0][1], labelled[0][2]
    for a, b, c, n in labelled[1:]:
        if a > end:
            g = a - end
            gaps[(endc, c)] += g
            gapn[n] += g
            sizes["< 10 us" if g < 1e4 else "10-100 us" if g < 1e5 else "0.1-1 ms" if g < 1e6 else ">= 1 ms"] += g
        if b > end:
            end, endc = b, c
    tot = sum(gaps.values())
    print(f"  idle gaps: {tot / 1e6:.1f} ms; by size: " + ", ".join(f"{k} {v / 1e6:.1f} ms" for k, v in sizes.most_common()))
    for (x, y), g in gaps.most_common():
        print(f"     {x:8s} -> {y:8s} {g / 1e6:8.1f} ms ({100 * g / max(1, tot):5.1f} %)")
    print("  idle before (next kernel):")
    for n, g in gapn.most_common(8):
        print(f"     {g / 1e6:8.1f} ms  {n[:70]}")


if __name__ == "__main__":
    main()
