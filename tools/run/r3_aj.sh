# Round 3: the trimmed 16-stream full-size batched parity test, then the whole GPU suite timed
# as the driver runs it (-q, no durations)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu > gpurun_out/r3aj_test.log 2>&1
echo rc=$?
