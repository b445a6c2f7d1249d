# three-plane k_gemmf on 16 waves (4 per SIMD) vs 8: kbench over M, the planes / tiny / full
# suites under it, C2 A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 20 > gpurun_out/r5q_kbench_gemmf_wr3.txt 2>&1 || { tail -20 gpurun_out/r5q_kbench_gemmf_wr3.txt; exit 1; }
VOX_HIP_GEMMF_WR3=4 timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm_planes.py tests/test_gpu_tiny.py tests/test_gpu_full.py::test_full_jfk_transcription tests/test_gpu_full.py::test_full_long_clip_one_shot > gpurun_out/r5q_test.log 2>&1 || { tail -40 gpurun_out/r5q_test.log; exit 1; }
tail -2 gpurun_out/r5q_test.log
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5q_c2_w2_$k.json 2> gpurun_out/r5q_err.txt || { tail -20 gpurun_out/r5q_err.txt; exit 1; }
  VOX_HIP_GEMMF_WR3=4 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5q_c2_w4_$k.json 2> gpurun_out/r5q_err.txt || { tail -20 gpurun_out/r5q_err.txt; exit 1; }
done
for f in gpurun_out/r5q_c2_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('prefill_ms'))"; done
echo rc=0
