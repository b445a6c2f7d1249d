# wo L2 warm-up beside the decode attention in the step graph: A/B on C2 (alternating), tests
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_WO_WARM=1 timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_full.py::test_full_jfk_transcription > gpurun_out/r5p_test.log 2>&1 || { tail -40 gpurun_out/r5p_test.log; exit 1; }
tail -2 gpurun_out/r5p_test.log
for k in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5p_c2_base$k.json 2> gpurun_out/r5p_err.txt || { tail -20 gpurun_out/r5p_err.txt; exit 1; }
  VOX_HIP_WO_WARM=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5p_c2_warm$k.json 2> gpurun_out/r5p_err.txt || { tail -20 gpurun_out/r5p_err.txt; exit 1; }
done
for f in gpurun_out/r5p_c2_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('decoder_ms_per_token'))"; done
echo rc=0
