# Round 3 final tree (after the cross-stream encoder pass): whole GPU suite, smoke(), every bench line, the served lines, the
# multi-rank path rehearsed on one GPU (2 ranks sharing it), and eager kernel stats of C2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --durations=20 --timeout 600 --timeout-method thread tests > gpurun_out/r3ai_test.log 2>&1 || { tail -30 gpurun_out/r3ai_test.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ai_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r3ai_bench.json 2> gpurun_out/r3ae.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --q8 > gpurun_out/r3ai_q8.json 2>> gpurun_out/r3ae.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r3ai_s16.json 2>> gpurun_out/r3ae.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 8 > gpurun_out/r3ai_s8.json 2>> gpurun_out/r3ae.err || exit 1
timeout -k 10 300 python -u bench.py --streams 16 --stagger --steps 1 --warmup 1 > gpurun_out/r3ai_serve16.json 2>> gpurun_out/r3ae.err || exit 1
timeout -k 10 300 python -u bench.py --streams 8 --stagger --steps 1 --warmup 1 > gpurun_out/r3ai_serve8.json 2>> gpurun_out/r3ae.err || exit 1
VOX_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3ai_gpus2_shared.json 2>> gpurun_out/r3ae.err || exit 1
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ai_prof_c2 -o c2 -- python3 -u bench.py --no-cpu-baseline --steps 2 > gpurun_out/r3ai_prof_c2.log 2>&1 || exit 1
echo rc=0
