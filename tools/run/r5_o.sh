# the 16-stream pre-encoded batched step's kernel table (eager launches: VOX_HIP_GRAPH=0)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5o_prof -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r5o_prof.log 2>&1 || { tail -20 gpurun_out/r5o_prof.log; exit 1; }
f=$(find gpurun_out/r5o_prof -name "*kernel_stats.csv" | head -1)
python3 tools/kstats.py "$f" 0 25
echo rc=0
