# Round 3, first box: the whole GPU suite incl. the new rolling-KV ring tests, the batched
# logit bar and the full-size -I 0.5 decode; then the contract bench line.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --durations=20 --timeout 400 --timeout-method thread tests > gpurun_out/r3a_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err
echo rc=$?
