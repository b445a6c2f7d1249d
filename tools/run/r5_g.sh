# scheduler test diagnosis (k_gemmf invalid argument in the bounded stacked prefill), then the
# C2 / 16-stream / served lines, then the k_gemmf unit-order sweep over M
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 250 --timeout-method thread tests/test_gpu_sched.py > gpurun_out/r5g_sched.log 2>&1
echo "sched rc=$?"; grep -E "passed|failed|Error" gpurun_out/r5g_sched.log | tail -5
timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r5g_c2.json 2> gpurun_out/r5g_err.txt || { tail -20 gpurun_out/r5g_err.txt; exit 1; }
timeout -k 10 240 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r5g_s16.json 2> gpurun_out/r5g_err.txt || { tail -20 gpurun_out/r5g_err.txt; exit 1; }
timeout -k 10 240 python -u bench.py --streams 8 --no-cpu-baseline > gpurun_out/r5g_s8.json 2> gpurun_out/r5g_err.txt || { tail -20 gpurun_out/r5g_err.txt; exit 1; }
for f in gpurun_out/r5g_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('decoder_ms_per_batched_step'), d.get('decoder_ms_per_token'))"; done
VOX_KB_ONLY=gemmf timeout -k 10 300 tools/kbench 20 > gpurun_out/r5g_kbench_gemmf.txt 2>&1 || { tail -20 gpurun_out/r5g_kbench_gemmf.txt; exit 1; }
echo rc=0
