# Round 3: k_attn_short (short-context decode attention without the state wait) -- kbench,
# parity (tiny, jfk full, twins, ring) and the contract bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 240 tools/kbench 200 | grep -E "attn decode|layer|gemv (qkv|wo|w13|w2)  " ) > gpurun_out/r3c_kb.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_twins.py tests/test_gpu_ring.py "tests/test_gpu_full.py::test_full_jfk_transcription" tests/test_gpu_attention.py > gpurun_out/r3c_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err && \
VOX_HIP_ATT_SHORT=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r3c_bench_old.json 2>> gpurun_out/r3c_bench.err
echo rc=$?
