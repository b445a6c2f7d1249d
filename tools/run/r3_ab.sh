# Round 3: batched wo with the residual folded in (k_sklx EPI_RESID, VOX_HIP_BATCH_WOX=1) on top
# of the fused W1|W3 + SwiGLU -- batched parity, A/B at 16 and 8 streams; kbench of the fused vs
# plain batched attention
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_BATCH_WOX=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_ring.py tests/test_gpu_sched.py > gpurun_out/r3ab_test.log 2>&1 || { tail -30 gpurun_out/r3ab_test.log; exit 1; }
for m in 1 0 1 0; do
  VOX_HIP_BATCH_WOX=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 16 > gpurun_out/r3ab_s16_$m.json 2>> gpurun_out/r3ab.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3ab_s16_$m.json'));print('s16 wox$m', d['value'], d['decoder_ms_per_batched_step'])"
  VOX_HIP_BATCH_WOX=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --streams 8 > gpurun_out/r3ab_s8_$m.json 2>> gpurun_out/r3ab.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3ab_s8_$m.json'));print('s8 wox$m', d['value'], d['decoder_ms_per_batched_step'])"
done
VOX_KB_ONLY=attb timeout -k 10 180 tools/kbench 100 > gpurun_out/r3ab_attb.txt 2>&1 || exit 1
# last (it may end in the profiler's SIGSEGV): the graph-replayed bench under the kernel trace
# with kernel arguments in host memory instead of device memory
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ab_graph -o g -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3ab_graph.log 2>&1
echo rc=$?
