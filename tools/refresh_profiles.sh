export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python bench.py > gpurun_out/r_b1.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --q8 > gpurun_out/r_q8.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 16 > gpurun_out/r_b16.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 8 > gpurun_out/r_b8.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline --streaming --steps 1 --warmup 1 > gpurun_out/r_b3.log 2>&1 &&
VOX_HIP_GRAPH=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/rprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/rprof.log 2>&1 &&
bash tools/pmc.sh
echo rc=$?
