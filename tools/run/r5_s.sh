# 16-stream full-size served parity (vs the single-stream path); decode GEMV per-block stamps
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_sched.py -k "16_streams" > gpurun_out/r5s_test.log 2>&1 || { tail -40 gpurun_out/r5s_test.log; exit 1; }
grep -E "passed|failed|stats" gpurun_out/r5s_test.log | tail -3
timeout -k 10 300 tools/kbench_stamps 5 > gpurun_out/r5s_kbench_stamps.txt 2>&1 || { tail -20 gpurun_out/r5s_kbench_stamps.txt; exit 1; }
grep -A2 "^stamps" gpurun_out/r5s_kbench_stamps.txt
echo rc=0
