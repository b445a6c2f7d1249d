# Round 3: the C host's per-GPU scheduler (tests + the staggered C4 serving line)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_sched.py > gpurun_out/r3b_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --streams 8 --stagger --steps 1 --warmup 1 > gpurun_out/r3b_serve8.json 2> gpurun_out/r3b_serve8.err && \
timeout -k 10 300 python -u bench.py --streams 16 --stagger --steps 1 --warmup 1 > gpurun_out/r3b_serve16.json 2> gpurun_out/r3b_serve16.err
echo rc=$?
