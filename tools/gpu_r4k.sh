# Batched residual + RMSNorm with all 18 w2 slabs in one load round: kbench row kernels,
# batch parity tests, 16-stream bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 150 tools/kbench 100 | grep -E "fplanes|swiglu" ) > gpurun_out/r4k_kb.log 2>&1 && \
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py > gpurun_out/r4k_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r4k_s16.json 2> gpurun_out/r4k.err
echo rc=$?
