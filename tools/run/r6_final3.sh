# Round 6 last tree check (after the prefill planes): the whole GPU suite, smoke, C2 bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r6final3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --durations=5 --timeout 600 --timeout-method thread tests > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d.get('encoder_rtf'), d.get('decoder_ms_per_token'), d['roofline']['frac'], d['cpu_baseline']['value'])"
echo rc=0
