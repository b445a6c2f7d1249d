# decode GEMV prologue: RMSNorm weights (and ada) loaded with x (one L2 round trip before the
# norm instead of two).  Parity (tiny, full jfk, Q8), then C2 and C5 alternating the new
# library with the previous one (tools/ab/libvoxtral_hip_base.so via VOX_HIP_LIB) on one box
# (tools/ab/libvoxtral_hip_base.so: the library built from the commit before the change, copied aside; not kept in the tree)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_q8.py tests/test_gpu_full.py -k "not long_clip and not 60s" > gpurun_out/r5i_test.log 2>&1 || { tail -30 gpurun_out/r5i_test.log; exit 1; }
tail -1 gpurun_out/r5i_test.log
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5i_$n.json 2> gpurun_out/r5i_err.txt || { tail -20 gpurun_out/r5i_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5i_$n.json')); print('$n', d['value'], d.get('decoder_ms_per_token'), d['roofline']['avg_launch_us'])"; }
for r in 1 2 3; do
VOX_HIP_LIB=tools/ab/libvoxtral_hip_base.so b c2_base_$r --no-cpu-baseline
b c2_new_$r --no-cpu-baseline
done
for r in 1 2; do
VOX_HIP_LIB=tools/ab/libvoxtral_hip_base.so b q8_base_$r --q8 --no-cpu-baseline
b q8_new_$r --q8 --no-cpu-baseline
done
VOX_KB_ONLY=none timeout -k 10 200 tools/kbench 100 > gpurun_out/r5i_kbench.txt 2>&1 || true
grep -E "^gemv (qkv|w13|lm)" gpurun_out/r5i_kbench.txt | head -20
echo rc=0
