# decode GEMVs with two groups in flight (PF): kbench sweep (bf16 + Q8), then the tiny/q8 suites
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemvpf timeout -k 10 300 tools/kbench 50 > gpurun_out/r5l_kbench_gemvpf.txt 2>&1 || { tail -20 gpurun_out/r5l_kbench_gemvpf.txt; exit 1; }
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_q8.py tests/test_gpu_gemm_planes.py > gpurun_out/r5l_test.log 2>&1 || { tail -40 gpurun_out/r5l_test.log; exit 1; }
tail -2 gpurun_out/r5l_test.log
timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r5l_c2.json 2> gpurun_out/r5l_err.txt || { tail -20 gpurun_out/r5l_err.txt; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5l_c2.json')); print(d['value'], d.get('encoder_rtf'), d.get('prefill_ms'), d['roofline']['avg_launch_us'])"
echo rc=0
