# Round 3: decode attention with the partial merge fused (last arriving block)
export TMPDIR=/tmp
mkdir -p gpurun_out
( VOX_KB_ONLY=attn timeout -k 5 120 tools/kbench 100 | grep attn ) > gpurun_out/r3l_attn.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_kv16.py tests/test_gpu_batch.py tests/test_gpu_twins.py tests/test_gpu_ring.py tests/test_gpu_tiny.py -s > gpurun_out/r3l_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --long-context 8192 > gpurun_out/r3l_long32.json 2> gpurun_out/r3l_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --long-context 8192 --kv-fp16 > gpurun_out/r3l_long16.json 2>> gpurun_out/r3l_bench.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3l_bench.json 2>> gpurun_out/r3l_bench.err
echo rc=$?
