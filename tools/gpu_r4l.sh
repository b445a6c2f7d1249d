# End-of-session check of the committed tree: full GPU suite and smoke()
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread tests > gpurun_out/r4l_test.log 2>&1 && \
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l_smoke.log 2>&1
echo rc=$?
