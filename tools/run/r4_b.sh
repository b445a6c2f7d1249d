# Round 4: step-capped serving (bursts ride in full batched steps), A/B against drain-every-run,
# kernel stats of the served line (eager) and a graph-replay profile attempt
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sched.py > gpurun_out/r4b_test.log 2>&1 || { tail -40 gpurun_out/r4b_test.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4b_serve16.json 2> gpurun_out/r4b.err || { tail -20 gpurun_out/r4b.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 --serve-step-cap 0 > gpurun_out/r4b_serve16_nocap.json 2>> gpurun_out/r4b.err || { tail -20 gpurun_out/r4b.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4b_serve8.json 2>> gpurun_out/r4b.err || { tail -20 gpurun_out/r4b.err; exit 1; }
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b_prof_serve16 -o serve16 -- python3 -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 40 > gpurun_out/r4b_prof_serve16.log 2>&1 || { tail -20 gpurun_out/r4b_prof_serve16.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b_prof_graph -o c2 -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r4b_prof_graph.log 2>&1 || { tail -30 gpurun_out/r4b_prof_graph.log; exit 1; }
echo rc=0
