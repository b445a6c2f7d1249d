# Multi-step decode graphs: bench line at 1 / 5 / 15 steps per graph, then the decode tests
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 5 15; do
  VOX_HIP_GRAPH_MULTI=$m timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4e_bench_m$m.json 2>> gpurun_out/r4e.err || exit 1
done
VOX_HIP_GRAPH_MULTI=5 timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r4e_q8_m5.json 2>> gpurun_out/r4e.err && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_full.py::test_full_jfk_transcription tests/test_gpu_tiny.py tests/test_gpu_batch.py tests/test_gpu_mel.py > gpurun_out/r4e_test.log 2>&1
echo rc=$?
