# Round 4 closing check: the whole GPU suite and smoke() on the final tree
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --durations=25 --timeout 400 --timeout-method thread tests > gpurun_out/r4z_test.log 2>&1 || { tail -40 gpurun_out/r4z_test.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z_smoke.txt 2>&1 || { tail -20 gpurun_out/r4z_smoke.txt; exit 1; }
tail -3 gpurun_out/r4z_test.log
echo rc=0
