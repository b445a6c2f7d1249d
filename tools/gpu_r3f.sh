export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 120 tools/kbench 100 | grep -E "^attn decode" ) > gpurun_out/r3f_kb.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_twins.py tests/test_gpu_attention.py tests/test_gpu_full.py::test_full_jfk_transcription > gpurun_out/r3f_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --streaming --audio-seconds 60 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r3f_stream.json 2> gpurun_out/r3f.err
echo rc=$?
