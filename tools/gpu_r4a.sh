# Round-2 re-entry check: full GPU suite, the contract bench line, GEMV kbench, and one SQ
# counter pass per GEMV flavour (bf16 / Q8) to settle whether the decode GEMVs are
# issue-bound or wait-bound.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 400 --timeout-method thread tests > gpurun_out/r4a_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err && \
( timeout -k 5 180 tools/kbench 100 | grep -E "gemv|occupancy" ) > gpurun_out/r4a_kb.log 2>&1 && \
VOX_HIP_GRAPH=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/r4a_sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r4a_sq.log 2>&1 && \
VOX_HIP_GRAPH=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/r4a_sqq8 -o run --output-format csv -- python3 bench.py --q8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r4a_sqq8.log 2>&1
echo rc=$?
