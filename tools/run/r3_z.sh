# Round 3 closing set (after the batched-row change): whole GPU suite, the bench lines of every
# config, C2's 5 s / 45 s clip lengths, and kernel stats of the 16-stream line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --durations=20 --timeout 400 --timeout-method thread tests > gpurun_out/r3z_test.log 2>&1 || { tail -30 gpurun_out/r3z_test.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r3z_bench.json 2> gpurun_out/r3z.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --q8 > gpurun_out/r3z_q8.json 2>> gpurun_out/r3z.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r3z_s16.json 2>> gpurun_out/r3z.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 8 > gpurun_out/r3z_s8.json 2>> gpurun_out/r3z.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --clip-seconds 5 > gpurun_out/r3z_clip5.json 2>> gpurun_out/r3z.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --clip-seconds 45 > gpurun_out/r3z_clip45.json 2>> gpurun_out/r3z.err || exit 1
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3z_prof_s16 -o s16 -- python3 -u bench.py --no-cpu-baseline --streams 16 --steps 2 > gpurun_out/r3z_prof_s16.log 2>&1 || exit 1
echo rc=0
