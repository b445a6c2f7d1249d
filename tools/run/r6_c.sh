# Round 6 call C: is the served encoder pass serialized with the batched steps by hardware-queue
# sharing?  Served 16 streams (graph replay) with GPU_MAX_HW_QUEUES 4 (default) / 8 / 16,
# alternated; eager kernel traces (short run) with 4 and 16 queues through tools/serve_timeline.py
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for r in 1 2; do
  b s16_q4_$r --stagger --streams 16 --no-cpu-baseline
  GPU_MAX_HW_QUEUES=8 b s16_q8_$r --stagger --streams 16 --no-cpu-baseline
  GPU_MAX_HW_QUEUES=16 b s16_q16_$r --stagger --streams 16 --no-cpu-baseline
done
for f in $O/s16_*.json; do python3 -c "import json; d=json.load(open('$f')); bd=d['batched_decode']; print('$f', d['value'], round(bd['ms']/bd['steps'],3), bd['rows_per_step'], d['tick_latency_ms'])"; done
export VOX_HIP_GRAPH=0
b s16_eager_q4 --stagger --streams 16 --no-cpu-baseline
GPU_MAX_HW_QUEUES=16 b s16_eager_q16 --stagger --streams 16 --no-cpu-baseline
for f in $O/s16_eager*.json; do python3 -c "import json; d=json.load(open('$f')); bd=d['batched_decode']; print('$f', d['value'], round(bd['ms']/bd['steps'],3))"; done
for qn in 4 16; do
  GPU_MAX_HW_QUEUES=$qn timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/tr$qn -o run --output-format csv -- python3 bench.py --stagger --streams 16 --steps 1 --warmup 0 --serve-seconds 40 --no-cpu-baseline > $O/tr$qn.log 2>&1 || { tail -20 $O/tr$qn.log; exit 1; }
  python3 tools/serve_timeline.py $(find /tmp/tr$qn -name "*kernel_trace.csv" | head -1) > $O/timeline16_q$qn.txt 2>&1; cat $O/timeline16_q$qn.txt
done
echo rc=0
