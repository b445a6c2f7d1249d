# decode GEMV prologue order: x (and the norm weights) issued before the first group's weights,
# so the row sum waits for x alone (B: Q8 keeps late norm-weight loads; C: Q8 early too), against
# the previous library (A); parity of B, then C2 and C5 alternating A / B / C on one box
# (tools/ab/libvoxtral_hip_base.so: the library built from the commit before the change, copied aside; not kept in the tree)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_q8.py tests/test_gpu_full.py -k "not long_clip and not 60s" > gpurun_out/r5k2_test.log 2>&1 || { tail -30 gpurun_out/r5k2_test.log; exit 1; }
VOX_HIP_LIB=tools/ab/libvoxtral_hip_c.so timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_q8.py > gpurun_out/r5k2_test_c.log 2>&1 || { tail -30 gpurun_out/r5k2_test_c.log; exit 1; }
tail -1 gpurun_out/r5k2_test.log gpurun_out/r5k2_test_c.log
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5k2_$n.json 2> gpurun_out/r5k2_err.txt || { tail -20 gpurun_out/r5k2_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5k2_$n.json')); print('$n', d['value'], d.get('decoder_ms_per_token'), d['roofline']['avg_launch_us'])"; }
for r in 1 2 3; do
VOX_HIP_LIB=tools/ab/libvoxtral_hip_base.so b c2_A_$r --no-cpu-baseline
b c2_B_$r --no-cpu-baseline
done
for r in 1 2; do
VOX_HIP_LIB=tools/ab/libvoxtral_hip_base.so b q8_A_$r --q8 --no-cpu-baseline
b q8_B_$r --q8 --no-cpu-baseline
VOX_HIP_LIB=tools/ab/libvoxtral_hip_c.so b q8_C_$r --q8 --no-cpu-baseline
done
echo rc=0
