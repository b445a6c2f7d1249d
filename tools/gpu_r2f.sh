# row-kernel changes: parity (tiny, batch, full), kbench, streaming + 16-stream bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_batch.py tests/test_gpu_attention.py tests/test_gpu_mel.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2f_test.log 2>&1 &&
timeout -k 10 120 tools/kbench 200 > gpurun_out/r2f_kbench.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --streaming --audio-seconds 60 --steps 1 --warmup 1 > gpurun_out/r2f_stream.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 16 --steps 2 --warmup 1 > gpurun_out/r2f_s16.log 2>&1
echo rc=$?
