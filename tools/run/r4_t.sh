# Round 4: k_attn_short late from wave 4 (keys 64..255) vs from wave 8 (default): parity with
# wave 4, C2 A/B on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_ATT_SHORT_LATE=4 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_attention.py tests/test_gpu_full.py::test_full_jfk_transcription > gpurun_out/r4t_test.log 2>&1 || { tail -40 gpurun_out/r4t_test.log; exit 1; }
for v in 4 8 4 8 4 8; do VOX_HIP_ATT_SHORT_LATE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r4t_c2_late$v.json 2>> gpurun_out/r4t.err || exit 1; echo "late$v $(cat gpurun_out/r4t_c2_late$v.json)" >> gpurun_out/r4t_c2_ab.txt; done
echo rc=0
