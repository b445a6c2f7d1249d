# k_sklx finisher: 16 slabs per load round (the streaming encoder's W2 finisher in one round);
# parity, then C3 (60 s, -I 0.5) alternating with the previous library on one box
# (tools/ab/libvoxtral_hip_base.so: the library built from the commit before the change, copied aside; not kept in the tree)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_full.py -k "encode or streaming or jfk" > gpurun_out/r5t_test.log 2>&1 || { tail -30 gpurun_out/r5t_test.log; exit 1; }
tail -1 gpurun_out/r5t_test.log
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > gpurun_out/r5t_$n.json 2> gpurun_out/r5t_err.txt || { tail -20 gpurun_out/r5t_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5t_$n.json')); print('$n', d['value'], d.get('encoder_ms_per_chunk'))"; }
for r in 1 2 3; do
VOX_HIP_LIB=tools/ab/libvoxtral_hip_base.so b st_A_$r --streaming --audio-seconds 60 --no-cpu-baseline
b st_B_$r --streaming --audio-seconds 60 --no-cpu-baseline
done
echo rc=0
