# Round 3: full-size batched parity at 8 and 16 streams (ids + last-step logits vs the oracle)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --durations=5 --timeout 600 --timeout-method thread tests/test_gpu_batch.py -k full_size > gpurun_out/r3ac_test.log 2>&1
echo rc=$?
