# Round-2 check: full -m gpu suite, smoke, default bench line.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_gputest.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1
echo rc=$?
