export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 120 tools/kbench 50 | grep -E "^gemm" ) > gpurun_out/r2u_kb3.log 2>&1 && \
( VOX_HIP_GEMM_PLANES=2 timeout -k 5 120 tools/kbench 50 | grep -E "^gemm" ) > gpurun_out/r2u_kb2.log 2>&1 && \
VOX_HIP_GEMM_PLANES=2 timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_full.py::test_full_jfk_transcription tests/test_gpu_full.py::test_full_long_clip_one_shot > gpurun_out/r2u_test2.log 2>&1
echo rc=$?
