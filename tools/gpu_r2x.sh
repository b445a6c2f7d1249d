export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r2x_bench.json 2> gpurun_out/r2x.err && \
timeout -k 10 300 python -u bench.py --clip-seconds 59.75 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r2x_clip.json 2>> gpurun_out/r2x.err && \
VOX_HIP_GEMM_PLANES=3 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r2x_bench3.json 2>> gpurun_out/r2x.err
echo rc=$?
