# Round-2 measurement pass: default bench line (config 2 + cpu baseline) and a rocprofv3
# kernel-stats profile of the streaming encoder (config 3, 60 s of audio, eager launches).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1 &&
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/sprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streaming --audio-seconds 60 --steps 1 --warmup 1 > gpurun_out/sprof.log 2>&1
echo rc=$?
