# Round 4 final: k_attn_short late from wave 4 by default -- the whole GPU suite, smoke, C2 / Q8
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread tests > gpurun_out/r4u_test.log 2>&1 || { tail -40 gpurun_out/r4u_test.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4u_smoke.txt 2>&1 || { tail -20 gpurun_out/r4u_smoke.txt; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r4u_bench.json 2> gpurun_out/r4u.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --q8 > gpurun_out/r4u_q8.json 2>> gpurun_out/r4u.err || exit 1
echo rc=0
