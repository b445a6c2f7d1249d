export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2l_prof -o run --output-format csv -- python3 bench.py --streaming --audio-seconds 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2l_stream.json 2> gpurun_out/r2l_stream.err
echo rc=$?
