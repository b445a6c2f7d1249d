export TMPDIR=/tmp
mkdir -p gpurun_out
VOX_HIP_ENC_FUSED=0 timeout -k 10 300 python -u bench.py --streams 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2o_s16_unfused.json 2> gpurun_out/r2o_s16.err && \
VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2o_prof -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2o_s16p.json 2>> gpurun_out/r2o_s16.err && \
VOX_HIP_ENC_FUSED=0 VOX_HIP_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2o_prof0 -o run --output-format csv -- python3 bench.py --streams 16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2o_s16p0.json 2>> gpurun_out/r2o_s16.err
echo rc=$?
