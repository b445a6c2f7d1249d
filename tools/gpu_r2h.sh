export TMPDIR=/tmp
mkdir -p gpurun_out
( timeout -k 5 60 tools/pstep_dbg 26 150 0 16 ) > gpurun_out/r2h_dbg.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pstep.py > gpurun_out/r2h_test.log 2>&1
echo rc=$?
