# Round 3: the rocprofv3 crash on the graph path with the graph packet capture off
export TMPDIR=/tmp
mkdir -p gpurun_out
DEBUG_HIP_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3r_graph -o g -- python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3r_graph.log 2>&1
echo rc=$?
