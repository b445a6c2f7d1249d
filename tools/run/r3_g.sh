# Round 3: k_gemmf with half-stage software pipeline -- diagnostics, encoder parity, bench
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=gemmf timeout -k 5 120 tools/kbench 100 | grep gemmf ) > gpurun_out/r3g_full.log 2>&1 && \
( VOX_KB_ONLY=gemmf timeout -k 5 120 tools/kbench_gfd1 100 | grep gemmf ) > gpurun_out/r3g_nomfma.log 2>&1 && \
( VOX_KB_ONLY=gemmf timeout -k 5 120 tools/kbench_gfd2 100 | grep gemmf ) > gpurun_out/r3g_nodma.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_gemm_planes.py tests/test_gpu_twins.py tests/test_gpu_mel.py "tests/test_gpu_full.py::test_full_jfk_transcription" "tests/test_gpu_full.py::test_full_long_clip_one_shot" > gpurun_out/r3g_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3g_bench.json 2> gpurun_out/r3g_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --clip-seconds 59.75 --steps 2 > gpurun_out/r3g_clip59.json 2>> gpurun_out/r3g_bench.err
echo rc=$?
