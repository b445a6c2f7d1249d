# the batched lines on the final tree: 16 / 8 pre-encoded streams, 16 served
export TMPDIR=/tmp
mkdir -p gpurun_out
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r5y_$n.json 2> gpurun_out/r5y_err.txt || { tail -20 gpurun_out/r5y_err.txt; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5y_$n.json')); print('$n', d['value'], d.get('decoder_ms_per_batched_step'))"; }
b s16 --streams 16 --no-cpu-baseline
b s8 --streams 8 --no-cpu-baseline
b serve16 --stagger --streams 16 --no-cpu-baseline
b q8 --q8 --no-cpu-baseline
echo rc=0
