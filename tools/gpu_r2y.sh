export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 32 80; do
VOX_HIP_ENC_SKINNY_ROWS=$r timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r2y_bench_$r.json 2>> gpurun_out/r2y.err || exit 1
done
VOX_HIP_ENC_SKINNY_ROWS=80 timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_full.py::test_full_jfk_transcription tests/test_gpu_tiny.py > gpurun_out/r2y_test.log 2>&1
echo rc=$?
