# k_gemmf owner with a parallel flag poll: small-M sweep of the least stages per block; the
# scheduler suite after the CU-share removal; C2 eager kernel table (rocprof)
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmfm timeout -k 10 300 tools/kbench 20 > gpurun_out/r5k_kbench_gemmfm.txt 2>&1 || { tail -20 gpurun_out/r5k_kbench_gemmfm.txt; exit 1; }
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_sched.py tests/test_gpu_gemm_planes.py tests/test_gpu_tiny.py > gpurun_out/r5k_test.log 2>&1 || { tail -40 gpurun_out/r5k_test.log; exit 1; }
tail -2 gpurun_out/r5k_test.log
timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r5k_c2.json 2> gpurun_out/r5k_err.txt || { tail -20 gpurun_out/r5k_err.txt; exit 1; }
VOX_HIP_ENC_SKINNY_ROWS=64 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r5k_c2_sk64.json 2> gpurun_out/r5k_err.txt || { tail -20 gpurun_out/r5k_err.txt; exit 1; }
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k_prof_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5k_prof_c2.log 2>&1 || { tail -20 gpurun_out/r5k_prof_c2.log; exit 1; }
for f in gpurun_out/r5k_c2*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('encoder_rtf_2plane'), d.get('prefill_ms'))"; done
find gpurun_out/r5k_prof_c2 -name "*kernel_stats.csv"
echo rc=0
