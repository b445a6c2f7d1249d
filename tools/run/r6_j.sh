# Round 6 call J: the decode attention inside the QKV GEMV launch
# (EPI_QKV_ATT).  Parity first (fused-attention test, full-size jfk / Q8, ring, kv16), then C2
# and Q8 alternated with VOX_HIP_ATT_FUSE=0 / 1 on one box, then a graph-replay kernel table
export TMPDIR=/tmp
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_attn_fused.py tests/test_gpu_full.py tests/test_gpu_q8.py tests/test_gpu_kv16.py tests/test_gpu_ring.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed|fused QKV" $O/test.log | tail -6
for i in 1 2; do
  for f in 0 1; do
    VOX_HIP_ATT_FUSE=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_f${f}_$i.json 2> $O/c2_f${f}_$i.err || { tail -20 $O/c2_f${f}_$i.err; exit 1; }
    VOX_HIP_ATT_FUSE=$f timeout -k 10 300 python -u bench.py --q8 --no-cpu-baseline > $O/q8_f${f}_$i.json 2> $O/q8_f${f}_$i.err || { tail -20 $O/q8_f${f}_$i.err; exit 1; }
  done
done
for f in $O/c2_*.json $O/q8_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d.get('decoder_ms_per_token'))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_full -o run --output-format csv -- python3 tools/graph_prof_py.py full > $O/prof_full.log 2>&1 || { tail -20 $O/prof_full.log; exit 1; }
python3 tools/kstats.py /tmp/prof_full/run_kernel_stats.csv > $O/graph_replay_kernels.txt 2>&1; head -12 $O/graph_replay_kernels.txt
echo rc=0
