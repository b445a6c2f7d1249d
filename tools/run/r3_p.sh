# Round 3: GEMV tail L2 prefetch of the next GEMV's first row groups -- parity + A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_twins.py tests/test_gpu_q8.py "tests/test_gpu_full.py::test_full_jfk_transcription" tests/test_gpu_kv16.py > gpurun_out/r3p_test.log 2>&1 && \
VOX_HIP_GEMV_PF=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3p_pf0.json 2> gpurun_out/r3p.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3p_pf1.json 2>> gpurun_out/r3p.err && \
VOX_HIP_GEMV_PF=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --q8 > gpurun_out/r3p_q8_pf0.json 2>> gpurun_out/r3p.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --q8 > gpurun_out/r3p_q8_pf1.json 2>> gpurun_out/r3p.err && \
VOX_HIP_GEMV_PF=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3p_pf0b.json 2>> gpurun_out/r3p.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3p_pf1b.json 2>> gpurun_out/r3p.err
echo rc=$?
