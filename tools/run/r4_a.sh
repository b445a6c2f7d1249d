# Round 4: device slot table for the batched decode (no re-capture on set changes, per-slot
# drop-out, one readback per chunk, batched prefills, alternatives in the batch)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --durations=10 --timeout 400 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_sched.py tests/test_gpu_full.py::test_full_gemmf_recompute_backstop_bit_identical > gpurun_out/r4a_test.log 2>&1 || { tail -40 gpurun_out/r4a_test.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4a_serve16.json 2> gpurun_out/r4a.err || { tail -20 gpurun_out/r4a.err; exit 1; }
timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r4a_s16.json 2>> gpurun_out/r4a.err || { tail -20 gpurun_out/r4a.err; exit 1; }
echo rc=0
