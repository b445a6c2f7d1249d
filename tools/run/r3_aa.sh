# Round 3: batched W1|W3 with the SwiGLU folded in (k_sklx tickets, VOX_HIP_BATCH_SWX=1) --
# batched parity, then A/B at 16 and 8 streams
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_BATCH_SWX=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_ring.py tests/test_gpu_sched.py > gpurun_out/r3aa_test.log 2>&1 || { tail -30 gpurun_out/r3aa_test.log; exit 1; }
for m in 1 0 1 0; do
  VOX_HIP_BATCH_SWX=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r3aa_s16_$m.json 2>> gpurun_out/r3aa.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3aa_s16_$m.json'));print('s16 swx$m', d['value'], d['decoder_ms_per_batched_step'])"
  VOX_HIP_BATCH_SWX=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 8 > gpurun_out/r3aa_s8_$m.json 2>> gpurun_out/r3aa.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3aa_s8_$m.json'));print('s8 swx$m', d['value'], d['decoder_ms_per_batched_step'])"
done
echo rc=0
