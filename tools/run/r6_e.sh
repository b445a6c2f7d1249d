# Round 6 call E: the served overlap -- batch queue at high vs normal priority (served 16,
# graph replay, alternated), and eager traces of both with the kernel sequence of the first
# step spans that contain encoder kernels (tools/serve_timeline.py --dump)
export TMPDIR=/tmp
O=gpurun_out/r6e; mkdir -p $O
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for r in 1 2; do
  b s16_hi_$r --stagger --streams 16 --no-cpu-baseline
  VOX_HIP_BATCH_PRIORITY=0 b s16_lo_$r --stagger --streams 16 --no-cpu-baseline
done
for f in $O/s16_*.json; do python3 -c "import json; d=json.load(open('$f')); bd=d['batched_decode']; print('$f', d['value'], round(bd['ms']/bd['steps'],3), bd['rows_per_step'], d['tick_latency_ms'])"; done
export VOX_HIP_GRAPH=0
for pr in 1 0; do
  VOX_HIP_BATCH_PRIORITY=$pr timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/trp$pr -o run --output-format csv -- python3 bench.py --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 20 --no-cpu-baseline > $O/trp$pr.log 2>&1 || { tail -20 $O/trp$pr.log; exit 1; }
  python3 tools/serve_timeline.py $(find /tmp/trp$pr -name "*kernel_trace.csv" | head -1) --dump > $O/timeline_prio$pr.txt 2>&1; head -30 $O/timeline_prio$pr.txt
done
echo rc=0
