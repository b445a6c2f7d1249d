export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r2t_bench.json 2> gpurun_out/r2t.err && \
timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r2t_q8.json 2>> gpurun_out/r2t.err && \
timeout -k 10 300 python -u bench.py --streaming --audio-seconds 60 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2t_stream60.json 2>> gpurun_out/r2t.err && \
timeout -k 10 300 python -u bench.py --streams 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2t_s16.json 2>> gpurun_out/r2t.err && \
timeout -k 10 300 python -u bench.py --streams 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2t_s8.json 2>> gpurun_out/r2t.err && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2t_prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2t_profbench.json 2>> gpurun_out/r2t.err
echo rc=$?
