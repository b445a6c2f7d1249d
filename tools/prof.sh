export TMPDIR=/tmp; export VOX_HIP_GRAPH=0
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1; echo rc=$?
