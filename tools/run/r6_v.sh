# Round 6 call V: the batched attention's grid at 32 rows -- one 1024-thread block per (stream,
# kv head) (default at >= 256 blocks) vs the 128-key block pairs (VOX_HIP_ATT_BSPLIT=2):
# batch tests under the forced split, then C4 32 streams pre-encoded alternated, and served
export TMPDIR=/tmp
O=gpurun_out/r6v; mkdir -p $O
VOX_HIP_ATT_BSPLIT=2 timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py -k "32 or full" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -3
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
for i in 1 2; do
  b s32_one_$i --streams 32 --no-cpu-baseline
  VOX_HIP_ATT_BSPLIT=2 b s32_split_$i --streams 32 --no-cpu-baseline
done
b serve32_one --stagger --streams 32 --no-cpu-baseline
VOX_HIP_ATT_BSPLIT=2 b serve32_split --stagger --streams 32 --no-cpu-baseline
for f in $O/s*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d.get('decoder_ms_per_batched_step'))"; done
echo rc=0
