# Round-6 closing lines (second pass, after the served / batched changes of DESIGN 16.11-16.14) on the final tree: GPU suite, smoke, every bench config (incl. the
# 32-stream lines), PMC traffic of the decode GEMVs (profiles/pmc_w13_traffic.json, read by
# bench.py), graph-replay kernel tables of the C2 decode and the batched step
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r6end2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --durations=10 --timeout 600 --timeout-method thread tests > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }; }
b bench
b s16 --streams 16 --no-cpu-baseline
b s32 --streams 32 --no-cpu-baseline
b s8 --streams 8 --no-cpu-baseline
b serve16 --stagger --streams 16 --no-cpu-baseline
b serve32 --stagger --streams 32 --no-cpu-baseline
b serve8 --stagger --streams 8 --no-cpu-baseline
b q8 --q8 --no-cpu-baseline
b kv16 --kv-fp16 --no-cpu-baseline
b stream60 --streaming --audio-seconds 60 --no-cpu-baseline
b clip59 --clip-seconds 59.75 --no-cpu-baseline
b long8192 --long-context 8192 --no-cpu-baseline
for f in $O/*.json; do echo $f; python3 -c "import json; d=json.load(open('$f')); print(d['value'], d.get('encoder_rtf'), d.get('decoder_ms_per_token'), d.get('decoder_ms_per_batched_step'))"; done
export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc_w13_traffic.json > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt | head -12
unset VOX_HIP_GRAPH
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_full -o run --output-format csv -- python3 tools/graph_prof_py.py full > $O/prof_full.log 2>&1 || { tail -20 $O/prof_full.log; exit 1; }
rm -f $O/pmc_fetch/*kernel_trace.csv $O/pmc_write/*kernel_trace.csv $O/prof_full/*kernel_trace.csv
echo rc=0
