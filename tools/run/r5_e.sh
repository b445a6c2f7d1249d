# scheduler tests (drain, CU shares), k_gemmf unit order over M, served 16 streams with CU shares
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_sched.py tests/test_gpu_tiny.py tests/test_gpu_batch.py tests/test_gpu_full.py tests/test_gpu_kv16.py > gpurun_out/r5e_test.log 2>&1 || { tail -40 gpurun_out/r5e_test.log; exit 1; }
tail -2 gpurun_out/r5e_test.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r5e_c2.json 2>gpurun_out/r5e_c2_err.txt || exit 1
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 20 > gpurun_out/r5e_kbench_gemmf.txt 2>&1 || { tail -20 gpurun_out/r5e_kbench_gemmf.txt; exit 1; }
for cfg in 0 96 128 96all; do
  case $cfg in
    96all) E="VOX_HIP_SCHED_ENC_CUS=96 VOX_HIP_SCHED_BATCH_ALL_CUS=1";;
    0b) E="VOX_HIP_SCHED_ENC_CUS=0";;
    *) E="VOX_HIP_SCHED_ENC_CUS=$cfg";;
  esac
  env $E timeout -k 10 300 python -u bench.py --stagger --streams 16 --no-cpu-baseline > gpurun_out/r5e_serve16_$cfg.json 2> gpurun_out/r5e_serve_err.txt || { tail -20 gpurun_out/r5e_serve_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5e_serve16_$cfg.json')); print('$cfg', d['value'], d['batched_decode']['ms']/d['batched_decode']['steps'], d['tick_latency_ms'])"
done
VOX_KB_ONLY=q8rb timeout -k 10 300 tools/kbench 50 > gpurun_out/r5e_kbench_q8rb.txt 2>&1 || { tail -20 gpurun_out/r5e_kbench_q8rb.txt; exit 1; }
grep gemv gpurun_out/r5e_kbench_q8rb.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e_prof_fullbatch -o run --output-format csv -- python3 tools/graph_prof_py.py fullbatch > gpurun_out/r5e_prof_fullbatch.log 2>&1 || { tail -20 gpurun_out/r5e_prof_fullbatch.log; exit 1; }
tail -1 gpurun_out/r5e_prof_fullbatch.log
echo rc=0
