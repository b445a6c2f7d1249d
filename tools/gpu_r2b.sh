# kbench (all decode / skinny / attention kernels) + rocprof kernel stats of the streaming encoder run
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 tools/kbench 200 > gpurun_out/r2_kbench.log 2>&1 &&
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streaming --audio-seconds 30 --steps 1 --warmup 1 > gpurun_out/r2_sprof.log 2>&1
echo rc=$?
