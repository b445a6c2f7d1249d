# Round 4: k_attn_short from wave 2 (VOX_HIP_ATT_SHORT_LATE=2) against the default from wave 4,
# C2 alternating; the attention/decode GPU tests under LATE=2; then the whole suite + smoke
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --no-cpu-baseline"
for i in 1 2 3; do
  for L in 4 2; do
    VOX_HIP_ATT_SHORT_LATE=$L timeout -k 10 200 $B >> gpurun_out/r4late2_c2_L$L.json 2>> gpurun_out/r4late2.err || { tail -20 gpurun_out/r4late2.err; exit 1; }
  done
done
VOX_HIP_ATT_SHORT_LATE=2 timeout -k 10 600 python -u -m pytest -m gpu -x -v -k "attn or decode or stream" --timeout 400 --timeout-method thread tests > gpurun_out/r4late2_test_L2.log 2>&1 || { tail -40 gpurun_out/r4late2_test_L2.log; exit 1; }
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --durations=25 --timeout 400 --timeout-method thread tests > gpurun_out/r4late2_test.log 2>&1 || { tail -40 gpurun_out/r4late2_test.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4late2_smoke.txt 2>&1 || { tail -20 gpurun_out/r4late2_smoke.txt; exit 1; }
tail -3 gpurun_out/r4late2_test_L2.log
tail -3 gpurun_out/r4late2_test.log
echo rc=0
