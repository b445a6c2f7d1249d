export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 120 tools/kbench 50 | grep -E "^gemm" ) > gpurun_out/r3e_kb.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_full.py tests/test_gpu_tiny.py tests/test_gpu_twins.py tests/test_gpu_gemm_planes.py tests/test_gpu_q8.py > gpurun_out/r3e_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3e_bench.json 2> gpurun_out/r3d.err && \
timeout -k 10 300 python -u bench.py --clip-seconds 59.75 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r3e_clip.json 2>> gpurun_out/r3d.err
echo rc=$?
