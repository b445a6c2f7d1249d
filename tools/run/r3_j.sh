# Round 3: gemmf tile choice + 16-bit decoder KV mode + long-context decode lines
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=gemmf timeout -k 5 120 tools/kbench 100 | grep gemmf ) > gpurun_out/r3j_gemmf.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_kv16.py tests/test_gpu_tiny.py tests/test_gpu_batch.py tests/test_gpu_twins.py tests/test_gpu_gemm_planes.py "tests/test_gpu_full.py::test_full_jfk_transcription" "tests/test_gpu_full.py::test_full_long_clip_one_shot" -s > gpurun_out/r3j_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3j_bench.json 2> gpurun_out/r3j_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --long-context 8192 > gpurun_out/r3j_long32.json 2>> gpurun_out/r3j_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --long-context 8192 --kv-fp16 > gpurun_out/r3j_long16.json 2>> gpurun_out/r3j_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --kv-fp16 > gpurun_out/r3j_bench16.json 2>> gpurun_out/r3j_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --clip-seconds 59.75 --steps 2 > gpurun_out/r3j_clip59.json 2>> gpurun_out/r3j_bench.err
echo rc=$?
