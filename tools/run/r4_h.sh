# Round 4: the scheduler's encoder pass beside the batched steps (vox_hip_batch_decode_rows,
# priority batch queue, batch-owned prefill workspace): scheduler / batch / tiny parity with
# the overlap on (default) and off, served lines A/B; kbench gemmf tile shapes and k_skl sweep
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sched.py tests/test_gpu_batch.py tests/test_gpu_tiny.py > gpurun_out/r4h_test.log 2>&1 || { tail -40 gpurun_out/r4h_test.log; exit 1; }
VOX_HIP_SCHED_OVERLAP=0 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sched.py -k "not full_size" > gpurun_out/r4h_test_ov0.log 2>&1 || { tail -40 gpurun_out/r4h_test_ov0.log; exit 1; }
B="python -u bench.py --no-cpu-baseline"
for ov in 1 0 1 0; do VOX_HIP_SCHED_OVERLAP=$ov timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4h_serve16_ov$ov.json 2>> gpurun_out/r4h.err || exit 1; echo "ov$ov $(cat gpurun_out/r4h_serve16_ov$ov.json)" >> gpurun_out/r4h_serve16_ab.txt; done
for ov in 1 0; do VOX_HIP_SCHED_OVERLAP=$ov timeout -k 10 300 $B --stagger --streams 8 --steps 1 --warmup 1 > gpurun_out/r4h_serve8_ov$ov.json 2>> gpurun_out/r4h.err || exit 1; done
VOX_KB_ONLY=sklks timeout -k 10 200 tools/kbench 100 > gpurun_out/r4h_kb_sklks.txt 2>&1 || { tail -20 gpurun_out/r4h_kb_sklks.txt; exit 1; }
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 50 > gpurun_out/r4h_kb_gemmf.txt 2>&1 || { tail -20 gpurun_out/r4h_kb_gemmf.txt; exit 1; }
echo rc=0
