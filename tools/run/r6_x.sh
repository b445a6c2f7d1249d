# Round 6 call X: the encoder attention writes the wo planes itself (no k_split_fplanes launch
# per layer when the keys are not split) vs the round-5 split (VOX_HIP_ATT_PLANES=0): encoder /
# planes / scheduler tests, then C2 (encoder RTF) and served 16 streams alternated
export TMPDIR=/tmp
O=gpurun_out/r6x; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_full.py tests/test_gpu_gemm_planes.py tests/test_gpu_twins.py tests/test_gpu_sched.py tests/test_gpu_kv16.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for i in 1 2; do
  VOX_HIP_ATT_PLANES=0 b c2_old_$i --no-cpu-baseline
  b c2_new_$i --no-cpu-baseline
done
VOX_HIP_ATT_PLANES=0 b clip_old --clip-seconds 59.75 --no-cpu-baseline
b clip_new --clip-seconds 59.75 --no-cpu-baseline
VOX_HIP_ATT_PLANES=0 b s16_old --stagger --streams 16 --no-cpu-baseline
b s16_new --stagger --streams 16 --no-cpu-baseline
for f in $O/c2_*.json $O/clip_*.json $O/s16_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d.get('encoder_rtf'), d.get('encoder_rtf_2plane'))"; done
echo rc=0
