"""Per-chunk GPU time of the streaming encoder's layer kernels from a rocprofv3
kernel_stats.csv (developer tool): chunks = k_attn_mf calls / encoder layers."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
layers = int(sys.argv[2]) if len(sys.argv) > 2 else 32
keys = ("k_sklx", "k_skl<", "k_attn_mf", "k_attn_tiled_combine", "k_rmsnorm_fplanes", "k_resid_rmsnorm_fplanes",
        "k_swiglu_fplanes", "k_slabs_rope_kv", "k_rmsnorm_rows")
chunks = sum(int(r["Calls"]) for r in rows if "k_attn_mf" in r["Name"]) / layers
tot = 0.0
for r in rows:
    if any(k in r["Name"] for k in keys) and "k_skl<" not in r["Name"] or ("k_skl<" in r["Name"]):
        if any(k in r["Name"] for k in keys):
            t = float(r["TotalDurationNs"]) / 1e3 / chunks
            tot += t
            print(f"  {r['Name'][:60]:60s} {t:8.1f} us/chunk  avg {float(r['AverageNs'])/1e3:7.2f}")
print(f"chunks {chunks:.0f}: encoder layer kernels {tot / 1e3:.3f} ms per chunk")
