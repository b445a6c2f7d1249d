"""Per-launch HBM traffic of the decode kernels from the two PMC passes of tools/pmc.sh.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (rocprofv3 derived counters).  On gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md
"HBM"), so reads are doubled; WRITE_SIZE is taken as reported.  Writes
profiles/pmc_w13_traffic.json (read by bench.py for roofline.traffic) and prints a table.

usage: python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write [out.json]
"""
import collections
import csv
import json
import os
import sys

W13 = "k_gemv<2, 4, 4, 2, 0>"   # PRO_NORM_ADA, EPI_SWIGLU, RB 4, KQ 2, bf16
W13_Q8 = "k_gemv<2, 4, 4, 1, 1>"  # the same, Q8 rows (int8 + f32 row scales)
ALGO = {  # algorithmic bytes per launch (weights + activation vectors), DESIGN.md section 5
    "k_gemv<2, 4, 4, 2, 0>": 2 * 9216 * 3072 * 2 + 3072 * 4 * 3 + 9216 * 4,
    "k_gemv<0, 1, 2, 5, 0>": 3072 * 9216 * 2 + 9216 * 4 + 3072 * 8,
    "k_gemv<1, 5, 4, 2, 0>": 6144 * 3072 * 2 + 3072 * 8 + 6144 * 4,
    "k_gemv<0, 1, 2, 2, 0>": 3072 * 4096 * 2 + 4096 * 4 + 3072 * 8,
    "k_gemv<1, 6, 8, 2, 0>": 131072 * 3072 * 2 + 3072 * 8 + 131072 * 4,
    # Q8 (config 5): int8 rows + f32 row scales
    "k_gemv<2, 4, 4, 1, 1>": 2 * 9216 * 3072 + 2 * 9216 * 4 + 3072 * 4 * 3 + 9216 * 4,
    "k_gemv<0, 1, 2, 3, 1>": 3072 * 9216 + 3072 * 4 + 9216 * 4 + 3072 * 8,
    "k_gemv<1, 5, 4, 1, 1>": 6144 * 3072 + 6144 * 4 + 3072 * 8 + 6144 * 4,
    "k_gemv<0, 1, 2, 1, 1>": 3072 * 4096 + 3072 * 4 + 4096 * 4 + 3072 * 8,
    "k_gemv<1, 6, 8, 1, 1>": 131072 * 3072 + 131072 * 4 + 3072 * 8 + 131072 * 4,
    # streaming encoder chunk (config 3, 25 rows = 2 row blocks of 16; the weights once):
    # QKV 6144 x 1280, W1|W3 10240 x 1280; <0, 4, 8> serves wo 1280 x 2048 and W2 1280 x 5120
    # (one template instance: their mean); planes and slabs are a few percent on top
    "k_skl<0, 4, 4>": 6144 * 1280 * 2,
    "k_skl<0, 8, 4>": 10240 * 1280 * 2,
    "k_skl<0, 4, 8>": (1280 * 2048 * 2 + 1280 * 5120 * 2) // 2,
}


def load(d, counter):
    f = os.path.join(d, "run_counter_collection.csv")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].replace("void vox::", "").replace("vox::", "").split("(")[0]
            agg[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_w13_traffic.json")
    fetch, n = load(fd, "FETCH_SIZE")
    write, _ = load(wd, "WRITE_SIZE")
    table = {}
    for k in sorted(fetch, key=lambda k: -fetch[k] * n[k]):
        rd = 2 * fetch[k] * 1024
        wr = write.get(k, 0.0) * 1024
        table[k] = {"launches": n[k], "read_bytes": round(rd), "write_bytes": round(wr),
                    "algorithmic_bytes": ALGO.get(k), "ratio": round((rd + wr) / ALGO[k], 4) if k in ALGO else None}
        print(f"{k:40s} n={n[k]:6d} read {rd / 1e6:9.2f} MB write {wr / 1e6:7.3f} MB"
              + (f"  algo {ALGO[k] / 1e6:8.2f} MB  ratio {table[k]['ratio']}" if k in ALGO else ""))
    key = W13 if W13 in table else W13_Q8
    w = table[key]
    res = {"kernel": key + " (W1|W3: RMSNorm*(1+ada) -> GEMV -> SiLU*up)",
           "hbm_bytes_per_launch": w["read_bytes"] + w["write_bytes"],
           "read_bytes_per_launch": w["read_bytes"], "write_bytes_per_launch": w["write_bytes"],
           "algorithmic_bytes_per_launch": ALGO[key], "launches": w["launches"],
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, eager decode "
                     "(tools/pmc.sh); FETCH_SIZE KiB x 1024 x 2 (gfx950 streaming-read correction)",
           "all_kernels": table}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
