# Round 6 call D: 32 slots per batched step (VOX_MAX_BATCH 32, VH_SCHED_MAX 32): batch /
# scheduler / tiny / ring GPU suites, then pre-encoded 16 / 32 streams and served 16 / 32
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_sched.py tests/test_gpu_tiny.py tests/test_gpu_ring.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
b s16 --streams 16 --no-cpu-baseline
b s32 --streams 32 --no-cpu-baseline
b serve16 --stagger --streams 16 --no-cpu-baseline
b serve32 --stagger --streams 32 --no-cpu-baseline
for f in $O/s16.json $O/s32.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['decoder_ms_per_batched_step'], d['encoder_rtf'])"; done
for f in $O/serve*.json; do python3 -c "import json; d=json.load(open('$f')); bd=d['batched_decode']; print('$f', d['value'], round(bd['ms']/bd['steps'],3), bd['rows_per_step'], d['tick_latency_ms'])"; done
echo rc=0
