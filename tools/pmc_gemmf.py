"""Per-projection PMC counters of the encoder's k_gemmf launches.

Reads one or more rocprofv3 --pmc runs (run_counter_collection.csv under each directory) of
the C2 bench with the decoder prefill off k_gemmf (VOX_HIP_PREFILL_GEMMF=0), so every k_gemmf
launch is an encoder projection of the one-shot pass.  Launches are labelled by epilogue and
order inside a layer: EPI 0 = QKV, EPI 4 = W1|W3, EPI 1 alternates wo / W2.  Prints, per
projection, the mean of each counter per launch; FETCH_SIZE is shown as bytes (KiB x 1024,
doubled for gfx950 streaming reads, MI355X_MICROARCH.md "HBM") next to the algorithmic bytes
(planes of the padded rows + bf16 weights) of the M rows given.
usage: python3 tools/pmc_gemmf.py M DIR [DIR ...]
"""
import collections
import csv
import os
import sys

ENC = {"QKV": (6144, 1280), "wo": (1280, 2048), "W1|W3": (10240, 1280), "W2": (1280, 5120)}  # N, K


def algo_bytes(name, M):
    N, K = ENC[name]
    mp = (M + 63) // 64 * 64  # 64-row tiles (three planes)
    return mp * K * 6 + N * K * 2


def main():
    M = int(sys.argv[1])
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[2:]:
        rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
        disp = collections.OrderedDict()
        for r in rows:
            n = r["Kernel_Name"]
            if "k_gemmf" not in n:
                continue
            key = (int(r["Dispatch_Id"]), n)
            disp.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
            disp[key]["_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        resid = 0
        for (did, n), c in sorted(disp.items()):
            targs = [t.strip() for t in n.split("k_gemmf<")[1].split(">")[0].split(",")]
            if targs[1] != "3":
                continue  # the bench's extra two-plane pass (encoder_rtf_2plane)
            epi = targs[0]
            if epi == "0":
                lab = "QKV"
            elif epi == "4":
                lab = "W1|W3"
            else:
                lab = "wo" if resid % 2 == 0 else "W2"
                resid += 1
            for k, v in c.items():
                vals[lab][k].append(v)
    for lab in ("QKV", "wo", "W1|W3", "W2"):
        if lab not in vals:
            continue
        c = vals[lab]
        n = max(len(v) for v in c.values())
        line = f"{lab:6s} n={n:4d}"
        for k in sorted(c):
            m = sum(c[k]) / len(c[k])
            if k == "FETCH_SIZE":
                b = 2 * m * 1024
                line += f"  fetch {b / 1e6:8.1f} MB ({b / algo_bytes(lab, M):5.2f}x of {algo_bytes(lab, M) / 1e6:.1f} MB algorithmic)"
            elif k == "_us":
                line += f"  {m:7.1f} us (under the profiler)"
            else:
                line += f"  {k} {m:,.0f}"
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h = sum(c["TCC_HIT_sum"]) / len(c["TCC_HIT_sum"])
            mi = sum(c["TCC_MISS_sum"]) / len(c["TCC_MISS_sum"])
            line += f"  L2 hit rate {h / max(1.0, h + mi):.3f}"
        print(line)


if __name__ == "__main__":
    main()
