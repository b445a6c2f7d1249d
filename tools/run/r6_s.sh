# Round 6 call S: the batched encoder pass's conv stems stacked on the lead's queue (one
# GEMM per conv for every stream, enc_prefix_batch) vs one stem per stream
# (VOX_HIP_ENC_STEM_BATCH=0): the batched-encoder / scheduler / mel parity tests, then served
# 16 / 32 streams alternated, then the eager trace's encoder kernel list
export TMPDIR=/tmp
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 800 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_tiny.py tests/test_gpu_sched.py tests/test_gpu_mel.py tests/test_gpu_full.py -k "encode or sched or mel or streaming or Scheduler or scheduler" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for i in 1 2; do
  VOX_HIP_ENC_STEM_BATCH=0 b s16_old_$i --stagger --streams 16 --no-cpu-baseline
  b s16_new_$i --stagger --streams 16 --no-cpu-baseline
done
VOX_HIP_ENC_STEM_BATCH=0 b s32_old --stagger --streams 32 --no-cpu-baseline
b s32_new --stagger --streams 32 --no-cpu-baseline
VOX_HIP_ENC_STEM_BATCH=0 b s8_old --stagger --streams 8 --no-cpu-baseline
b s8_new --stagger --streams 8 --no-cpu-baseline
for f in $O/s*.json; do python3 -c "import json; d=json.load(open('$f')); bd=d['batched_decode']; print('$f', d['value'], round(bd['ms']/bd['steps'],3), bd['rows_per_step'], d['tick_latency_ms'])"; done
export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/trn -o run --output-format csv -- python3 bench.py --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 20 --no-cpu-baseline > $O/trn.log 2>&1 || { tail -20 $O/trn.log; exit 1; }
python3 tools/serve_timeline.py $(find /tmp/trn -name "*kernel_trace.csv" | head -1) --top 16 > $O/timeline.txt 2>&1; head -6 $O/timeline.txt; grep -A17 "encoder: top" $O/timeline.txt
echo rc=0
