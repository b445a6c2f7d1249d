# Kernel stats of the batched decode (config 4, 16 streams) and of the Q8 line (config 5)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c_s16 -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r4c_s16.log 2>&1 && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c_q8 -o run --output-format csv -- python3 bench.py --q8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r4c_q8.log 2>&1
echo rc=$?
