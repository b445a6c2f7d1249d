# k_gemmw (weights in registers): kbench check + sweep against k_gemmf, then the encoder /
# prefill GPU tests with VOX_HIP_GEMMW=1
export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_KB_ONLY=gemmw timeout -k 10 300 tools/kbench 20 > gpurun_out/r5i_kbench_gemmw.txt 2>&1 || { tail -20 gpurun_out/r5i_kbench_gemmw.txt; exit 1; }
grep check gpurun_out/r5i_kbench_gemmw.txt
VOX_HIP_GEMMW=1 timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm_planes.py tests/test_gpu_tiny.py tests/test_gpu_full.py > gpurun_out/r5i_test.log 2>&1 || { tail -40 gpurun_out/r5i_test.log; exit 1; }
tail -2 gpurun_out/r5i_test.log
VOX_HIP_GEMMW=1 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r5i_c2_gemmw.json 2> gpurun_out/r5i_err.txt || { tail -20 gpurun_out/r5i_err.txt; exit 1; }
timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r5i_c2.json 2> gpurun_out/r5i_err.txt || { tail -20 gpurun_out/r5i_err.txt; exit 1; }
for f in gpurun_out/r5i_c2*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('encoder_rtf_2plane'), d.get('prefill_ms'))"; done

VOX_HIP_SCHED_ENC_CUS=96 VOX_HIP_SCHED_BATCH_ALL_CUS=1 timeout -k 10 300 python -u bench.py --stagger --streams 16 --no-cpu-baseline > gpurun_out/r5i_serve16_96all.json 2> gpurun_out/r5i_serve_err.txt || { tail -20 gpurun_out/r5i_serve_err.txt; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r5i_serve16_96all.json')); print('96all', d['value'], d['batched_decode']['ms']/d['batched_decode']['steps'], d.get('tick_latency_ms'))"
echo rc=0
