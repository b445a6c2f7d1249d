# Three-wave GEMVs where the row's chunks are a multiple of 192: kbench (NW4 vs auto), decode
# parity tests, bf16 and Q8 bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 150 tools/kbench 100 | grep -E "gemv|occupancy" ) > gpurun_out/r4h_kb.log 2>&1 && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_q8.py tests/test_gpu_full.py::test_full_jfk_transcription tests/test_gpu_twins.py > gpurun_out/r4h_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r4h_bench.json 2> gpurun_out/r4h.err && \
timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > gpurun_out/r4h_q8.json 2>> gpurun_out/r4h.err
echo rc=$?
