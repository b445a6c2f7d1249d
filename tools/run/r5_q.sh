# k_resid_xw_fplanes: every slab of the batched step's wo / W2 in one round of loads (24 per
# round instead of 8); batch parity, then 16 / 8 pre-encoded streams alternating with the
# previous library (tools/ab/libvoxtral_hip_base.so, VOX_HIP_LIB) on one box
# (tools/ab/libvoxtral_hip_base.so: the library built from the commit before the change, copied aside; not kept in the tree)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_sched.py > gpurun_out/r5q_test.log 2>&1 || { tail -30 gpurun_out/r5q_test.log; exit 1; }
tail -1 gpurun_out/r5q_test.log
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5q_$n.json 2> gpurun_out/r5q_err.txt || { tail -20 gpurun_out/r5q_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5q_$n.json')); print('$n', d['value'], d.get('decoder_ms_per_batched_step'))"; }
for r in 1 2 3; do
VOX_HIP_LIB=tools/ab/libvoxtral_hip_base.so b s16_A_$r --streams 16 --no-cpu-baseline
b s16_B_$r --streams 16 --no-cpu-baseline
done
VOX_HIP_LIB=tools/ab/libvoxtral_hip_base.so b s8_A --streams 8 --no-cpu-baseline
b s8_B --streams 8 --no-cpu-baseline
echo rc=0
