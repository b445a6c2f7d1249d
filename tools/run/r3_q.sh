# Round 3: rocprofv3 kernel trace of the graph-replayed decode (the product path)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3q_graph -o g -- python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3q_graph.log 2>&1
echo rc=$?
