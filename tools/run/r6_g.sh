# Round 6 call G: the scheduler submits the batched steps before the encoder pass
# (vox_hip_batch_begin_rows / finish) -- scheduler + batch suites, then served 16 and 32
# streams with the new order vs the round-5 order (VOX_HIP_SCHED_STEPS_FIRST=0), alternated,
# and an eager trace of the new order (kernel sequence of the first step spans with encoder kernels)
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_sched.py tests/test_gpu_batch.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -2
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for r in 1 2; do
  b s16_new_$r --stagger --streams 16 --no-cpu-baseline
  VOX_HIP_SCHED_STEPS_FIRST=0 b s16_old_$r --stagger --streams 16 --no-cpu-baseline
done
b s32_new --stagger --streams 32 --no-cpu-baseline
VOX_HIP_SCHED_STEPS_FIRST=0 b s32_old --stagger --streams 32 --no-cpu-baseline
for f in $O/s*.json; do python3 -c "import json; d=json.load(open('$f')); bd=d['batched_decode']; print('$f', d['value'], round(bd['ms']/bd['steps'],3), bd['rows_per_step'], d['tick_latency_ms'])"; done
export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/trn -o run --output-format csv -- python3 bench.py --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 20 --no-cpu-baseline > $O/trn.log 2>&1 || { tail -20 $O/trn.log; exit 1; }
python3 tools/serve_timeline.py $(find /tmp/trn -name "*kernel_trace.csv" | head -1) --dump > $O/timeline_new.txt 2>&1; head -16 $O/timeline_new.txt
echo rc=0
