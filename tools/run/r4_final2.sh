# Round 4: the default bench line and the served 16-stream line on the final library build
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r4f2_bench.json 2> gpurun_out/r4f2.err || { tail -20 gpurun_out/r4f2.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --stagger --streams 16 --steps 1 --warmup 1 > gpurun_out/r4f2_serve16.json 2>> gpurun_out/r4f2.err || { tail -20 gpurun_out/r4f2.err; exit 1; }
echo rc=0
