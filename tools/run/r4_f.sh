# Round 4: attention merge factors per thread (no second barrier) + 4-row readlane reductions:
# parity (batch, attention, tiny, ring), phase stamps, and an A/B of this build against the
# r4_c build (ab/libvoxtral_hip_d53.so, VOX_HIP_LIB) on one box: 16 / 8 streams and C2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_attention.py tests/test_gpu_tiny.py tests/test_gpu_ring.py > gpurun_out/r4f_test.log 2>&1 || { tail -40 gpurun_out/r4f_test.log; exit 1; }
VOX_KB_ONLY=attb timeout -k 10 200 tools/kbench 100 > gpurun_out/r4f_kb_attb.txt 2>&1 || { tail -20 gpurun_out/r4f_kb_attb.txt; exit 1; }
B="python -u bench.py --no-cpu-baseline"
for v in new old new old; do
  if [ $v = old ]; then export VOX_HIP_LIB=ab/libvoxtral_hip_d53.so; else unset VOX_HIP_LIB; fi
  timeout -k 10 200 $B --streams 16 > gpurun_out/r4f_s16_$v.json 2>> gpurun_out/r4f.err || exit 1; echo "$v $(cat gpurun_out/r4f_s16_$v.json)" >> gpurun_out/r4f_s16_ab.txt
  timeout -k 10 200 $B --streams 8 > gpurun_out/r4f_s8_$v.json 2>> gpurun_out/r4f.err || exit 1; echo "$v $(cat gpurun_out/r4f_s8_$v.json)" >> gpurun_out/r4f_s8_ab.txt
  timeout -k 10 200 $B --steps 10 --warmup 2 > gpurun_out/r4f_c2_$v.json 2>> gpurun_out/r4f.err || exit 1; echo "$v $(cat gpurun_out/r4f_c2_$v.json)" >> gpurun_out/r4f_c2_ab.txt
done
unset VOX_HIP_LIB
echo rc=0
