export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_tiny.py > gpurun_out/r2n_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --streams 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2n_s16.json 2> gpurun_out/r2n_s16.err
echo rc=$?
