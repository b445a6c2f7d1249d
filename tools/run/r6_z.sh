# Round 6 call Z: PMC traffic of the 32-row batched step (FETCH_SIZE / WRITE_SIZE in separate
# passes, eager), tools/pmc_summary.py per kernel
export TMPDIR=/tmp
O=gpurun_out/r6z; mkdir -p $O
export VOX_HIP_GRAPH=0
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/pf32 -o run --output-format csv -- python3 bench.py --streams 32 --steps 1 --warmup 0 --no-cpu-baseline > $O/pf.log 2>&1 || { tail -20 $O/pf.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/pw32 -o run --output-format csv -- python3 bench.py --streams 32 --steps 1 --warmup 0 --no-cpu-baseline > $O/pw.log 2>&1 || { tail -20 $O/pw.log; exit 1; }
python3 tools/pmc_summary.py /tmp/pf32 /tmp/pw32 $O/pmc32.json > $O/pmc32.txt 2>&1; head -24 $O/pmc32.txt
echo rc=0
