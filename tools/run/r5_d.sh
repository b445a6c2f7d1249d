# C3 streaming (-I 0.5) encoder chunks: kernel table and dispatch gaps (eager launches), to
# split a 25-row chunk's 2.07 ms between kernel time and launch boundaries
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5d_prof -o run -- python3 bench.py --streaming --audio-seconds 20 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5d_prof.log 2>&1 || { tail -20 gpurun_out/r5d_prof.log; exit 1; }
db=$(find gpurun_out/r5d_prof -name "*results.db" | head -1)
python3 tools/db_stats.py "$db" 40 gaps > gpurun_out/r5d_stats.txt
python3 - "$db" > gpurun_out/r5d_chunks.txt <<'PY'
import sqlite3, sys
db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()
# encoder chunk windows: from a k_im2col3 (conv stem) to the next decoder GEMV / the end
enc = ("k_sklx", "k_attn", "k_im2col3", "k_gemmf", "k_skl", "k_rope", "k_gemm", "k_rmsnorm", "k_split", "k_conv", "k_mel", "k_adapt", "k_gelu")
chunks = []
cur = None
for name, st, en in rows:
    short = name.split("(")[0].replace("void vox::", "")
    if short.startswith("k_im2col3"):
        if cur: chunks.append(cur)
        cur = [st, en, 0, 0]
    if cur is not None and not short.startswith("k_gemv") and not short.startswith("k_argmax") and not short.startswith("k_attn_short"):
        cur[1] = max(cur[1], en); cur[2] += en - st; cur[3] += 1
    elif cur is not None and (short.startswith("k_gemv") or short.startswith("k_argmax")):
        chunks.append(cur); cur = None
if cur: chunks.append(cur)
print("# chunk windows (conv stem .. next decoder kernel): wall us, sum of kernel us, kernels")
for c in chunks[:200]:
    print(f"{(c[1]-c[0])/1e3:9.1f} {c[2]/1e3:9.1f} {c[3]:5d}")
import statistics
if chunks:
    w = [ (c[1]-c[0])/1e3 for c in chunks]; k = [c[2]/1e3 for c in chunks]
    print(f"# median wall {statistics.median(w):.1f} us, median kernel sum {statistics.median(k):.1f} us, n {len(chunks)}")
PY
tail -2 gpurun_out/r5d_chunks.txt
head -30 gpurun_out/r5d_stats.txt
echo rc=0
