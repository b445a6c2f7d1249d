export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_tiny.py tests/test_gpu_full.py::test_full_streaming_60s_encoder > gpurun_out/r2p_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --streams 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2p_s16.json 2> gpurun_out/r2p.err && \
timeout -k 10 300 python -u bench.py --streaming --audio-seconds 30 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2p_stream.json 2>> gpurun_out/r2p.err && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p_prof -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2p_s16p.json 2>> gpurun_out/r2p.err
echo rc=$?
