# Round 6 final tree check (after the encoder attention planes): GPU suite, smoke, C2 / Q8 / C4 16 and 32 / served 16 bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r6final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --durations=5 --timeout 600 --timeout-method thread tests > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
b bench
b q8 --q8 --no-cpu-baseline
b s16 --streams 16 --no-cpu-baseline
b s32 --streams 32 --no-cpu-baseline
b serve16 --stagger --streams 16 --no-cpu-baseline
b stream60 --streaming --audio-seconds 60 --no-cpu-baseline
for f in $O/*.json; do echo $f; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('decoder_ms_per_token'), d.get('decoder_ms_per_batched_step'), d.get('encoder_ms_per_chunk'))"; done
echo rc=0
