# Profiled batches with graph replays for all but the sampled step: bf16 and Q8 bench lines,
# plus the decode parity tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4d_bench.json 2> gpurun_out/r4d.err && \
timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r4d_q8.json 2>> gpurun_out/r4d.err && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_full.py::test_full_jfk_transcription tests/test_gpu_tiny.py tests/test_gpu_q8.py > gpurun_out/r4d_test.log 2>&1
echo rc=$?
