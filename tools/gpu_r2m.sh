export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py::test_encode_chunks_match tests/test_gpu_full.py::test_full_streaming_60s_encoder > gpurun_out/r2m_test.log 2>&1 && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2m_prof -o run --output-format csv -- python3 bench.py --streaming --audio-seconds 10 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2m_stream.json 2> gpurun_out/r2m_stream.err
echo rc=$?
