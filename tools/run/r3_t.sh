# Round 3 re-entry: the whole GPU suite on the restored tree, the contract bench line, then
# the rocprofv3 graph-replay reproduction (tiny graphs first, then the product bench).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --durations=20 --timeout 400 --timeout-method thread tests > gpurun_out/r3t_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r3t_bench.json 2> gpurun_out/r3t_bench.err && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t_prof0 -o r -- tools/graph_prof_repro 0 > gpurun_out/r3t_prof0.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t_prof1 -o r -- tools/graph_prof_repro 1 > gpurun_out/r3t_prof1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t_prof2 -o r -- tools/graph_prof_repro 2 > gpurun_out/r3t_prof2.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t_prof3 -o r -- tools/graph_prof_repro 3 > gpurun_out/r3t_prof3.log 2>&1
echo rc=$?
