# Round 6 call T: the batched LM head over 17..32 rows as one k_skf<Z = 2> launch (embeddings
# read once) vs one launch per 16-row block (VOX_HIP_SKF2=0): tools/kbench VOX_KB_ONLY=sknb
# (skf lines, bits compared), the batch tests, then C4 32 streams pre-encoded and served
export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
VOX_KB_ONLY=sknb timeout -k 10 300 tools/kb_run 100 > $O/kb_sknb.txt 2>&1 || { tail -20 $O/kb_sknb.txt; exit 1; }
grep -E "^skf" $O/kb_sknb.txt
timeout -k 10 700 python -u -m pytest -m gpu -x -v --timeout 600 --timeout-method thread tests/test_gpu_batch.py > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for i in 1 2; do
  VOX_HIP_SKF2=0 b s32_old_$i --streams 32 --no-cpu-baseline
  b s32_new_$i --streams 32 --no-cpu-baseline
done
VOX_HIP_SKF2=0 b serve32_old --stagger --streams 32 --no-cpu-baseline
b serve32_new --stagger --streams 32 --no-cpu-baseline
for f in $O/s*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d.get('decoder_ms_per_batched_step'))"; done
echo rc=0
