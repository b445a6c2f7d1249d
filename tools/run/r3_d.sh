# Round 3: k_gemmf (stream-K MFMA GEMM over planes x fragment-major weights) -- kbench at the
# encoder shapes, encoder parity (tiny chunks, planes modes, twins, full jfk / 59.75 s), bench
export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 300 tools/kbench 100 | grep -E "gemmf|gemm enc|gemm pre" ) > gpurun_out/r3d_kb.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_gemm_planes.py tests/test_gpu_twins.py tests/test_gpu_mel.py "tests/test_gpu_full.py::test_full_jfk_transcription" "tests/test_gpu_full.py::test_full_long_clip_one_shot" > gpurun_out/r3d_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --clip-seconds 59.75 --steps 2 > gpurun_out/r3d_clip59.json 2>> gpurun_out/r3d_bench.err
echo rc=$?
