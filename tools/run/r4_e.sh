# Round 4: the batched wo projection merging the decode attention's key-range partials
# (AttnFuse.wom, k_skl_attn): parity (batch / scheduler / tiny suites, wom on and off),
# attention + wo kbench A/B, pre-encoded and served lines A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_sched.py tests/test_gpu_tiny.py tests/test_gpu_ring.py > gpurun_out/r4e_test.log 2>&1 || { tail -40 gpurun_out/r4e_test.log; exit 1; }
VOX_HIP_BATCH_WOM=0 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_batch.py > gpurun_out/r4e_test_wom0.log 2>&1 || { tail -40 gpurun_out/r4e_test_wom0.log; exit 1; }
VOX_KB_ONLY=attb timeout -k 10 200 tools/kbench 100 > gpurun_out/r4e_kb_attb.txt 2>&1 || { tail -20 gpurun_out/r4e_kb_attb.txt; exit 1; }
B="python -u bench.py --no-cpu-baseline"
for w in 1 0 1 0; do VOX_HIP_BATCH_WOM=$w timeout -k 10 200 $B --streams 16 > gpurun_out/r4e_s16_wom$w.json 2>> gpurun_out/r4e.err || exit 1; cat gpurun_out/r4e_s16_wom$w.json >> gpurun_out/r4e_s16_ab.jsonl; done
for w in 1 0; do VOX_HIP_BATCH_WOM=$w timeout -k 10 200 $B --streams 8 > gpurun_out/r4e_s8_wom$w.json 2>> gpurun_out/r4e.err || exit 1; done
for w in 1 0; do VOX_HIP_BATCH_WOM=$w timeout -k 10 300 $B --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4e_serve16_wom$w.json 2>> gpurun_out/r4e.err || exit 1; done
echo rc=0
