export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_full.py::test_full_jfk_transcription tests/test_gpu_twins.py tests/test_gpu_q8.py tests/test_gpu_pstep.py > gpurun_out/r3b_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3b_bench.json 2> gpurun_out/r3b.err && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r3b_pb.json 2>> gpurun_out/r3b.err
echo rc=$?
