# encoder single-row GEMV path + batched QKV 6-block splits: encoder/batch GPU tests, C2 and C4 lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_full.py tests/test_gpu_batch.py tests/test_gpu_q8.py tests/test_gpu_twins.py > gpurun_out/r5c_test.log 2>&1 || { tail -40 gpurun_out/r5c_test.log; exit 1; }
tail -2 gpurun_out/r5c_test.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5c_c2.json 2>gpurun_out/r5c_err.txt || exit 1
timeout -k 10 200 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r5c_s16.json 2>gpurun_out/r5c_err.txt || exit 1
VOX_HIP_LIB=build/ab/libvoxtral_hip_r4.so VOX_HIP_GEMM_PLANES=3 timeout -k 10 200 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r5c_s16_r4.json 2>gpurun_out/r5c_err.txt || exit 1
VOX_HIP_LIB=build/ab/libvoxtral_hip_r4.so VOX_HIP_GEMM_PLANES=3 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5c_c2_r4.json 2>gpurun_out/r5c_err.txt || exit 1
for f in gpurun_out/r5c_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('decoder_ms_per_batched_step'))"; done
echo rc=0
