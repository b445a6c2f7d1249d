# HBM traffic of the decode kernels from PMC counters (MI355X_MICROARCH.md "HBM"):
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), eager decode steps
# (VOX_HIP_GRAPH=0), one short bench run each; summarised by tools/pmc_summary.py.
export TMPDIR=/tmp; export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
echo rc=$?
