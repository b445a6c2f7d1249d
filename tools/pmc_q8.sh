# HBM traffic of the Q8 decode kernels (config 5) from PMC counters: FETCH_SIZE and
# WRITE_SIZE in separate passes, eager decode steps; summarised by tools/pmc_summary.py into
# profiles/pmc_w13_q8_traffic.json.
export TMPDIR=/tmp; export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcq8_fetch -o run --output-format csv -- python3 bench.py --q8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcq8_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcq8_write -o run --output-format csv -- python3 bench.py --q8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcq8_write.log 2>&1
echo rc=$?
