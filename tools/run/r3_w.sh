# Round 3: batched projections cold / MALL-hot / warm head (touch kernel first); rocprofv3
# graph repro with dispatch-event launches interleaved (mode 5)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=skb timeout -k 10 180 tools/kbench 100 > gpurun_out/r3w_skb.txt 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3w_prof5 -o r -- tools/graph_prof_repro 5 > gpurun_out/r3w_prof5.log 2>&1
echo rc=$?
