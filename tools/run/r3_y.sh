# Round 3: batched step with slice-parallel residual + x*w planes (RMSNorm applied by the
# projection) -- kernel timings, batched parity tests, bench A/B at 16 and 8 streams
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=skb timeout -k 10 180 tools/kbench 100 > gpurun_out/r3y_skb.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_ring.py tests/test_gpu_sched.py tests/test_gpu_kv16.py > gpurun_out/r3y_test.log 2>&1 || { tail -30 gpurun_out/r3y_test.log; exit 1; }
for m in 1 0 1 0; do
  VOX_HIP_BATCH_XW=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r3y_s16_xw$m.json 2>> gpurun_out/r3y.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3y_s16_xw$m.json'));print('s16 xw$m', d['value'], d['decoder_ms_per_batched_step'])"
  VOX_HIP_BATCH_XW=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 8 > gpurun_out/r3y_s8_xw$m.json 2>> gpurun_out/r3y.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3y_s8_xw$m.json'));print('s8 xw$m', d['value'], d['decoder_ms_per_batched_step'])"
done
echo rc=0
