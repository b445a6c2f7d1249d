# Round 3: the async-encode API under interleaved streams (TINY, vs the oracle)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py > gpurun_out/r3af_test.log 2>&1
echo rc=$?
