# after the null-flags fix and the shape-picked k_gemmf unit order: full GPU suite, smoke, C2,
# served 16 streams with and without CU shares
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --durations=10 --timeout 400 --timeout-method thread tests > gpurun_out/r5h_test.log 2>&1 || { tail -40 gpurun_out/r5h_test.log; exit 1; }
tail -3 gpurun_out/r5h_test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5h_smoke.txt 2>&1 || { tail -20 gpurun_out/r5h_smoke.txt; exit 1; }
timeout -k 10 240 python -u bench.py > gpurun_out/r5h_bench.json 2> gpurun_out/r5h_bench.err || { tail -20 gpurun_out/r5h_bench.err; exit 1; }
VOX_HIP_GEMMF_ORDER=2 timeout -k 10 240 python -u bench.py --no-cpu-baseline > gpurun_out/r5h_c2_rowmajor.json 2> gpurun_out/r5h_err.txt || { tail -20 gpurun_out/r5h_err.txt; exit 1; }
for cfg in 0 96 96all; do
  VOX_HIP_SCHED_ENC_CUS=$cfg timeout -k 10 300 python -u bench.py --stagger --streams 16 --no-cpu-baseline > gpurun_out/r5h_serve16_$cfg.json 2> gpurun_out/r5h_serve_err.txt || { tail -20 gpurun_out/r5h_serve_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5h_serve16_$cfg.json')); print('$cfg', d['value'], d['batched_decode']['ms']/d['batched_decode']['steps'], d.get('tick_latency_ms'))"
done
for f in gpurun_out/r5h_bench.json gpurun_out/r5h_c2_rowmajor.json; do echo $f; python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('encoder_rtf_2plane'), d.get('prefill_ms'), d.get('decoder_ms_per_token'))"; done
echo rc=0
