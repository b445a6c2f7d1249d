export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 5 120 tools/kbench 100 > gpurun_out/r2j_kbench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --streaming --audio-seconds 30 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r2j_stream.json 2> gpurun_out/r2j_stream.err
echo rc=$?
