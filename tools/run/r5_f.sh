# Round 5, re-entry check of HEAD: full GPU suite, smoke, C2, 16/8-stream steps, served 16 streams
# with and without CU shares, rocprof of the 16-stream step
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --durations=10 --timeout 400 --timeout-method thread tests > gpurun_out/r5f_test.log 2>&1 || { tail -40 gpurun_out/r5f_test.log; exit 1; }
tail -3 gpurun_out/r5f_test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f_smoke.txt 2>&1 || { tail -20 gpurun_out/r5f_smoke.txt; exit 1; }
timeout -k 10 240 python -u bench.py > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || { tail -20 gpurun_out/r5f_bench.err; exit 1; }
timeout -k 10 240 python -u bench.py --streams 16 --no-cpu-baseline > gpurun_out/r5f_s16.json 2> gpurun_out/r5f_err.txt || { tail -20 gpurun_out/r5f_err.txt; exit 1; }
timeout -k 10 240 python -u bench.py --streams 8 --no-cpu-baseline > gpurun_out/r5f_s8.json 2> gpurun_out/r5f_err.txt || { tail -20 gpurun_out/r5f_err.txt; exit 1; }
for cfg in 0 96 128; do
  VOX_HIP_SCHED_ENC_CUS=$cfg timeout -k 10 300 python -u bench.py --stagger --streams 16 --no-cpu-baseline > gpurun_out/r5f_serve16_$cfg.json 2> gpurun_out/r5f_serve_err.txt || { tail -20 gpurun_out/r5f_serve_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5f_serve16_$cfg.json')); print('$cfg', d['value'], d['batched_decode']['ms']/d['batched_decode']['steps'], d.get('tick_latency_ms'))"
done
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_prof_s16 -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r5f_prof_s16.log 2>&1 || exit 1
for f in gpurun_out/r5f_*.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('decoder_ms_per_batched_step'), d.get('decoder_ms_per_token'))"; done
echo rc=0
