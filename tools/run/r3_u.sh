# Round 3: batched-decode kernel options (k_skl vs whole-K k_skf at 16 rows; fused batched
# attention by context and block split), then rocprofv3 kernel trace of the graph-replayed
# default bench (the product path; eager launches were profiled so far)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=skb timeout -k 10 180 tools/kbench 100 > gpurun_out/r3u_skb.txt 2>&1 && \
VOX_KB_ONLY=attb timeout -k 10 180 tools/kbench 100 > gpurun_out/r3u_attb.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3u_graph -o g -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3u_graph.log 2>&1
echo rc=$?
