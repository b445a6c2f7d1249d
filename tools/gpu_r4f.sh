# Round-2 closing measurement pass: every bench line, the default line's rocprofv3 kernel stats
# (graph replays traced), then the full GPU suite
export TMPDIR=/tmp
mkdir -p gpurun_out
# (rocprofv3 cannot follow graph replays: its hipGraphLaunch hook crashed, so the profiled run launches eagerly)
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4f_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r4f_prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r4f_q8.json 2>> gpurun_out/r4f.err && \
timeout -k 10 300 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r4f_s16.json 2>> gpurun_out/r4f.err && \
timeout -k 10 300 python -u bench.py --streams 8 --no-cpu-baseline > gpurun_out/r4f_s8.json 2>> gpurun_out/r4f.err && \
timeout -k 10 300 python -u bench.py --streaming --audio-seconds 60 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r4f_stream60.json 2>> gpurun_out/r4f.err && \
timeout -k 10 300 python -u bench.py --clip-seconds 59.75 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4f_clip59.json 2>> gpurun_out/r4f.err && \
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread tests > gpurun_out/r4f_test.log 2>&1
echo rc=$?
