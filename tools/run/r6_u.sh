# Round 6 call U: the batched W1|W3 over 17..32 rows as k_sklx2 (both row blocks per block,
# one ticket per slice) vs k_sklx's block per row block (VOX_HIP_SKLX2=0): batch + scheduler
# tests, then C4 32 streams pre-encoded and served, alternated; the 32-row step's kernel table
export TMPDIR=/tmp
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 800 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_sched.py -k "32 or full or batch" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for i in 1 2; do
  VOX_HIP_SKLX2=0 b s32_old_$i --streams 32 --no-cpu-baseline
  b s32_new_$i --streams 32 --no-cpu-baseline
done
VOX_HIP_SKLX2=0 b serve32_old --stagger --streams 32 --no-cpu-baseline
b serve32_new --stagger --streams 32 --no-cpu-baseline
for f in $O/s*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d.get('decoder_ms_per_batched_step'))"; done
export VOX_HIP_GRAPH=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p32 -o run --output-format csv -- python3 bench.py --streams 32 --steps 1 --warmup 0 --no-cpu-baseline > $O/p32.log 2>&1 || { tail -20 $O/p32.log; exit 1; }
python3 tools/kstats.py /tmp/p32/run_kernel_stats.csv > $O/s32_kernels.txt 2>&1; head -14 $O/s32_kernels.txt
echo rc=0
