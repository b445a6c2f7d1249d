# Round 5 first check: GPU suite on the slimmer library (hygiene, 3-plane default, scheduler drain),
# smoke, then the C2 and C4 bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread tests > gpurun_out/r5a_test.log 2>&1 || { tail -40 gpurun_out/r5a_test.log; exit 1; }
tail -3 gpurun_out/r5a_test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5a_smoke.txt 2>&1 || { tail -20 gpurun_out/r5a_smoke.txt; exit 1; }
timeout -k 10 240 python -u bench.py > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err || { tail -20 gpurun_out/r5a_bench.err; exit 1; }
timeout -k 10 240 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r5a_s16.json 2> gpurun_out/r5a_s16.err || { tail -20 gpurun_out/r5a_s16.err; exit 1; }
cat gpurun_out/r5a_bench.json gpurun_out/r5a_s16.json
echo rc=0
