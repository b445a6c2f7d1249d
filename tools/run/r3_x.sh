# Round 3: weight-head prefetch in the short decode attention (VOX_HIP_ATT_PF modes) --
# parity on the decode tests, then a bench A/B over the modes (bf16, then Q8)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_ATT_PF=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tiny.py "tests/test_gpu_full.py::test_full_jfk_transcription" tests/test_gpu_q8.py > gpurun_out/r3x_test.log 2>&1 || exit 1
for m in 0 1 2 3 4 0 2; do
  VOX_HIP_ATT_PF=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r3x_pf$m.json 2>> gpurun_out/r3x.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3x_pf$m.json'));print('bf16 pf$m', d['value'], d['decoder_ms_per_token'])"
done
for m in 0 2 1 0 2; do
  VOX_HIP_ATT_PF=$m timeout -k 10 200 python -u bench.py --no-cpu-baseline --q8 > gpurun_out/r3x_q8_pf$m.json 2>> gpurun_out/r3x.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3x_q8_pf$m.json'));print('q8 pf$m', d['value'], d['decoder_ms_per_token'])"
done
echo rc=0
