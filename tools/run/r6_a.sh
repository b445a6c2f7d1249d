# Round 6, first GPU call: (1) one 16-row batch vs two concurrent 8-row batches (tools/exp_dual.py);
# (2) PMC FETCH_SIZE / WRITE_SIZE of the 16-stream pre-encoded batched step (eager), separate passes
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 300 python -u tools/exp_dual.py 16 3 > $O/dual16.txt 2>&1 || { tail -30 $O/dual16.txt; exit 1; }
cat $O/dual16.txt
timeout -k 10 300 python -u tools/exp_dual.py 8 3 > $O/dual8.txt 2>&1 || { tail -30 $O/dual8.txt; exit 1; }
cat $O/dual8.txt
export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write $O/pmc16.json > $O/pmc16.txt 2>&1; head -30 $O/pmc16.txt
echo rc=0
