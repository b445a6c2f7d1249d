# Round 4 closing on the final tree (k_attn_short LATE by default): the whole GPU suite, smoke,
# and the C2 / Q8 / streaming / 16-stream lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread tests > gpurun_out/r4s_test.log 2>&1 || { tail -40 gpurun_out/r4s_test.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4s_smoke.txt 2>&1 || { tail -20 gpurun_out/r4s_smoke.txt; exit 1; }
B="timeout -k 10 300 python -u bench.py"
$B > gpurun_out/r4s_bench.json 2> gpurun_out/r4s.err || exit 1
$B --no-cpu-baseline --q8 > gpurun_out/r4s_q8.json 2>> gpurun_out/r4s.err || exit 1
$B --no-cpu-baseline --streaming --audio-seconds 60 --steps 1 --warmup 1 > gpurun_out/r4s_stream60.json 2>> gpurun_out/r4s.err || exit 1
$B --no-cpu-baseline --kv-fp16 > gpurun_out/r4s_c2_kv16.json 2>> gpurun_out/r4s.err || exit 1
echo rc=0
