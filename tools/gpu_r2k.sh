export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_full.py::test_full_streaming_60s_encoder tests/test_gpu_q8.py::test_q8_streaming_skinny_encoder_and_batch > gpurun_out/r2k_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --streaming --audio-seconds 30 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2k_stream.json 2> gpurun_out/r2k_stream.err
echo rc=$?
