# the final tree: full GPU suite, smoke, the default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --durations=10 --timeout 400 --timeout-method thread tests > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d.get('encoder_rtf'), d['roofline'], d['cpu_baseline'])"
echo rc=0
