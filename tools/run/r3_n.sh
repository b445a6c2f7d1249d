# Round 3: every config's bench line on the current tree + kernel stats of the batched step
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline --q8 > gpurun_out/r3n_q8.json 2> gpurun_out/r3n.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 8 > gpurun_out/r3n_s8.json 2>> gpurun_out/r3n.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r3n_s16.json 2>> gpurun_out/r3n.err && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline --streaming --audio-seconds 180 --steps 1 --warmup 0 > gpurun_out/r3n_stream180.json 2>> gpurun_out/r3n.err && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_prof_s16 -o s16 -- python -u bench.py --no-cpu-baseline --streams 16 --steps 2 > gpurun_out/r3n_prof_s16.log 2>&1 && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_prof_c2 -o c2 -- python -u bench.py --no-cpu-baseline --steps 2 > gpurun_out/r3n_prof_c2.log 2>&1
echo rc=$?
