# Round 3: the scheduler's deferred chunks through one batched encoder pass per run --
# scheduler / C host parity, then the served C4 line A/B (VOX_HIP_SCHED_BATCH_ENC=1 vs 0)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tiny.py "tests/test_gpu_full.py::test_full_encode_mel_batch_streaming_chunks" tests/test_gpu_sched.py tests/test_host_c.py > gpurun_out/r3ah_test.log 2>&1 || { tail -30 gpurun_out/r3ah_test.log; exit 1; }
for m in 1 0; do
  VOX_HIP_SCHED_BATCH_ENC=$m timeout -k 10 300 python -u bench.py --streams 16 --stagger --steps 1 --warmup 1 > gpurun_out/r3ah_serve16_$m.json 2>> gpurun_out/r3ah.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3ah_serve16_$m.json').read().strip().splitlines()[-1]);print('serve16 benc$m', d['value'], d['tick_latency_ms'], d['batched_decode'])"
  VOX_HIP_SCHED_BATCH_ENC=$m timeout -k 10 300 python -u bench.py --streams 8 --stagger --steps 1 --warmup 1 > gpurun_out/r3ah_serve8_$m.json 2>> gpurun_out/r3ah.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3ah_serve8_$m.json').read().strip().splitlines()[-1]);print('serve8 benc$m', d['value'], d['tick_latency_ms'], d['batched_decode'])"
done
echo rc=0
