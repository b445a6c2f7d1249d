# Round 6 call Y: the decoder prefill's attention writes the wo planes too (dec_layers_gemmf
# without its split launch): prefill / batch / scheduler / ring / kv16 / q8 suites, then served
# 16 streams alternated with VOX_HIP_ATT_PLANES=0 (both splits back)
export TMPDIR=/tmp
O=gpurun_out/r6y; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_full.py tests/test_gpu_tiny.py tests/test_gpu_batch.py tests/test_gpu_sched.py tests/test_gpu_kv16.py tests/test_gpu_q8.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for i in 1 2; do
  VOX_HIP_ATT_PLANES=0 b s16_old_$i --stagger --streams 16 --no-cpu-baseline
  b s16_new_$i --stagger --streams 16 --no-cpu-baseline
done
for f in $O/s16_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['tick_latency_ms'])"; done
echo rc=0
