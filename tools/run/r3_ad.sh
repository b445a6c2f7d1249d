# Round 3: scheduled streams' encoder chunks enqueued without a sync (several in flight) --
# scheduler parity, then the served C4 line A/B (VOX_HIP_SCHED_ASYNC=1 default vs 0)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sched.py tests/test_host_c.py > gpurun_out/r3ad_test.log 2>&1 || { tail -30 gpurun_out/r3ad_test.log; exit 1; }
for m in 1 0; do
  VOX_HIP_SCHED_ASYNC=$m timeout -k 10 300 python -u bench.py --streams 16 --stagger --steps 1 --warmup 1 > gpurun_out/r3ad_serve16_$m.json 2>> gpurun_out/r3ad.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3ad_serve16_$m.json').read().strip().splitlines()[-1]);print('serve16 async$m', d['value'], d['tick_latency_ms'], d['batched_decode'])"
  VOX_HIP_SCHED_ASYNC=$m timeout -k 10 300 python -u bench.py --streams 8 --stagger --steps 1 --warmup 1 > gpurun_out/r3ad_serve8_$m.json 2>> gpurun_out/r3ad.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3ad_serve8_$m.json').read().strip().splitlines()[-1]);print('serve8 async$m', d['value'], d['tick_latency_ms'], d['batched_decode'])"
done
echo rc=0
